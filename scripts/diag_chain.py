"""Diagnostic: is the in-kernel multi-pass chain bitwise == single passes, per config and kernel kind?"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raytracer-0_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np
import rt0, oracle as O
cfgs = O.load_configs()
for name in ["c2_cornell_mis_refcaps", "c2_cornell_mis_8", "c1_cornell_cos"]:
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    for jit in (True, False):
        r = rt0.Renderer(64, 64); r.set_jit(jit); rt0.configure(r, cfg, cfgs)
        r.render(1, 4); a = r.read_accum()
        r.clear(); r.render(1, 1); r.render(2, 1); r.render(3, 2); b = r.read_accum()
        r.clear(); r.render(1, 1); s1 = r.read_accum()
        r.clear(); r.render(1, 4); c = r.read_accum()
        print(name, "jit" if jit else "aot", "chain!=split: %.4f" % (a != b).any(-1).mean(),
              "rerun!=: %.4f" % (a != c).any(-1).mean(), "maxdiff %.3g" % np.abs(a - b).max(), flush=True)
