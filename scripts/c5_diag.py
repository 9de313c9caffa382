"""C5 cost split (diagnostic): the C5 pass kernel's time with the glass model,
with the model made diffuse white, and without the model, by kernel-trace
free HIP-event timing of one 4096^2 ReSTIR pass (min of 3 after 2 warm-up
passes).  python3 scripts/c5_diag.py"""
import copy
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

base = workloads.get("c5")
variants = {"glass": base}
w = copy.deepcopy(base)
w["scene_lines"] = [l.replace("MAT_SPECTRAL_FLINT", "MAT_WHITE") for l in w["scene_lines"]]
variants["diffuse_model"] = w
w = copy.deepcopy(base)
w["scene_lines"] = [l for l in w["scene_lines"] if "TRIANGLE" not in l]
w["models"] = []
variants["no_model"] = w
for name, wl in variants.items():
    r = rt0.Renderer(wl["width"], wl["height"])
    workloads.configure(r, wl)
    ts = []
    for k in range(1, 6):
        r.render(k, 1)
        if k > 2:
            ts.append(r.last_kernel_ms()[0])
    print(name, "ms per pass %.3f" % min(ts), r.last_render_path(), flush=True)
    r.close()
