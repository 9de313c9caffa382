#!/usr/bin/env python3
"""Kernel time of small launches (C1-sized images): where does a 256^2 x 16 spp
step spend its time?  Prints kernel ms per render() for a few shapes."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "raytracer-0_amd"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402  (configs.json loader only)
import rt0  # noqa: E402


def main():
    cfgs = O.load_configs()
    for name, w, spp in (("c1_cornell_cos", 256, 16), ("c1_cornell_cos", 256, 64), ("c1_cornell_cos", 1024, 16),
                         ("c2_cornell_mis_8", 256, 16), ("c2_cornell_mis_8", 1024, 16)):
        cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
        r = rt0.Renderer(w, w)
        rt0.configure(r, cfg, cfgs)
        r.render(1, spp)
        ks = []
        t0 = time.perf_counter()
        for s in range(5):
            r.render(1 + spp * (s + 1), spp)
            ks.append(r.last_kernel_ms())
        dt = (time.perf_counter() - t0) / 5
        print(json.dumps({"name": name, "w": w, "spp": spp, "kernel": ks[-1], "wall_ms": round(dt * 1e3, 3),
                          "Msamples_s": round(w * w * spp / dt / 1e6, 1)}), flush=True)
        r.close()


if __name__ == "__main__":
    main()
