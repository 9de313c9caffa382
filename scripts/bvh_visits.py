"""BVH node visits per walk on C5 (diagnostic; needs the probe build):
    PROBES_PATCH=scripts/probes_visits.patch scripts/probes.sh env \\
        RT0_JIT_EXTRA=-DRT0_EXP_VISITS python scripts/bvh_visits.py
(probes.sh applies $PROBES_PATCH to a scratch copy and builds it there).
Renders the BASELINE C5 workload's ReSTIR chain to pass 3, then counts pass 4:
histograms of nodes visited per walk, closest-hit walks (the pass kernel's
camera and bounce rays) by outcome -- no triangle, a triangle hit from
outside, from inside the model (a glass path's ray leaving it) -- and
occlusion walks (the walk kernel's visibility and shadow rays) unoccluded /
occluded.  `--compile-only` just builds the probe module (no GPU)."""
import json
import os
import sys

import ctypes

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

CLASSES = ["closest: no triangle", "closest: hit from outside", "closest: hit from inside",
           "occlusion: unoccluded", "occlusion: occluded"]
NC = 11 + 5 * 64 + 5

wl = workloads.get("c5")
if "--compile-only" in sys.argv:
    scene, sdf = rt0.scene_strings({"scene_lines": wl["scene_lines"], "sdf_kinds": wl.get("sdf_kinds", [])},
                                   {"cornell_lines": None})
    print("probe module bytes", rt0.jit_compile(scene, sdf, rt0.parse_config(
        *rt0.config_strings({"defines": wl["defines"], "constants": wl["constants"]}))))
    sys.exit(0)
r = rt0.Renderer(wl["width"], wl["height"])
workloads.configure(r, wl)
r.render(1, 3)
r.render(4, 1)
out = (ctypes.c_uint64 * NC)()
n = rt0.lib().rt0_read_counters_n(r.h, out, NC)
assert n == NC, ("not the probe build", n)
res = {}
for k, name in enumerate(CLASSES):
    h = [out[11 + 64 * k + b] for b in range(64)]
    walks = sum(h)
    total = out[11 + 320 + k]
    acc, pct = 0, {}
    for b, c in enumerate(h):  # bin b = [4b, 4b + 4) nodes (63: >= 252)
        acc += c
        for q in (50, 90, 99):
            if q not in pct and walks and acc >= q / 100.0 * walks:
                pct[q] = 4 * b + 3
    res[name] = {"walks": walks, "mean_nodes": total / max(1, walks), "p50_le": pct.get(50), "p90_le": pct.get(90),
                 "p99_le": pct.get(99), "share_of_nodes": None, "hist4": h}
    print("%-28s walks %10d  mean %6.1f nodes  p50 <= %s  p90 <= %s  p99 <= %s"
          % (name, walks, total / max(1, walks), pct.get(50), pct.get(90), pct.get(99)), flush=True)
allnodes = sum(out[11 + 320 + k] for k in range(5))
for k, name in enumerate(CLASSES):
    res[name]["share_of_nodes"] = out[11 + 320 + k] / max(1, allnodes)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/bvh_visits_c5.json", "w"), indent=1)
