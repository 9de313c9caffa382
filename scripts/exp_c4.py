"""A/B timing of the C4 workload's kernel under profiling-only macros
(RT0_JIT_EXTRA) and constant overrides, to see where its time goes.
usage: python scripts/exp_c4.py [size] [spp] [causes]
(the "causes" probes need the probe source: scripts/probes.sh python scripts/exp_c4.py 1024 8 causes)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wl = workloads.get("c4")
# (name, RT0_JIT_EXTRA, RT0_JIT_WAVES_PER_EU, constant overrides)
VARIANTS = [("budget16", "", "", {}), ("budget4", "-DRT0_MARCH_BUDGET=4", "", {}),
            ("budget8", "-DRT0_MARCH_BUDGET=8", "", {}), ("budget32", "-DRT0_MARCH_BUDGET=32", "", {}),
            ("budget128", "-DRT0_MARCH_BUDGET=128", "", {}), ("b8_w5", "-DRT0_MARCH_BUDGET=8", "5", {}),
            ("b8_w6", "-DRT0_MARCH_BUDGET=8", "6", {}), ("budget16", "", "", {})]
if len(sys.argv) > 3 and sys.argv[3] == "causes":
    VARIANTS = [("base", "", "", {}), ("no_vol_nee", "-DRT0_EXP_NO_VOL_NEE", "", {}),
                ("no_nee", "-DRT0_EXP_NO_NEE", "", {}), ("no_shadow", "-DRT0_EXP_NO_SHADOW", "", {}),
                ("march64", "", "", {"MARCHING_STEPS": 64}), ("march32", "", "", {"MARCHING_STEPS": 32})]
for name, extra, waves, consts in VARIANTS:
    os.environ["RT0_JIT_EXTRA"] = extra
    if waves:
        os.environ["RT0_JIT_WAVES_PER_EU"] = waves
    else:
        os.environ.pop("RT0_JIT_WAVES_PER_EU", None)
    r = rt0.Renderer(size, size)
    workloads.configure(r, wl, consts)
    r.render(1, 1)
    best = 1e30
    for k in range(3):
        r.render(2 + k * spp, spp)
        best = min(best, r.last_kernel_ms()[0])
    r.set_counting(True)
    r.render(1, 1)
    c = r.counters()
    r.set_counting(False)
    n = float(c["samples"]) if c["samples"] else 1.0
    print("%-12s %8.2f ms / %d spp at %d^2   isect/sample %.2f map/sample %.1f" %
          (name, best, spp, size, c["isect"] / n, c["map"] / n), flush=True)
    r.close()
