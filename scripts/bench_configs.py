#!/usr/bin/env python3
"""Msamples/s of the other BASELINE.json configurations on one MI355X.

bench.py measures configs[1] (C2, the headline).  This times C1 (256^2 Cornell,
4 bounces, cosine only), C3 (1920x1080 outdoor ReSTIR), C4 (2048^2 Mandelbulb +
homogeneous volume, 12 bounces) and C5 (spectral + ReSTIR/MIS + an 81,920-
triangle model through the LBVH) on a single GPU, one JSON line per config:
wall-clock Msamples/s of rt0_render over `spp` passes (scene resident, JIT
compiled and BVH built during the warm-up) and the kernels' own HIP-event time.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "raytracer-0_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as O  # noqa: E402  (configs.json loader only)
import rt0  # noqa: E402
from rt0 import meshes as M  # noqa: E402

# name, width, height, passes per step, constant overrides
RUNS = {
    "c1": ("c1_cornell_cos", 256, 256, 16, {}),
    "c3": ("c3_outdoor_restir", 1920, 1080, 16, {}),
    "c4": ("c4_mandelbulb_vol", 2048, 2048, 8, {"MAX_BOUNCES": 12}),
    "c5": ("c5_spectral_models", 4096, 4096, 4, {}),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", default="c1,c3,c4,c5")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    cfgs = O.load_configs()
    for key in args.runs.split(","):
        name, w, h, spp, over = RUNS[key]
        cfg = dict([c for c in cfgs["configs"] if c["name"] == name][0])
        cfg["constants"] = dict(cfg.get("constants", {}), **over)
        r = rt0.Renderer(w, h)
        rt0.configure(r, cfg, cfgs)
        for k, m in enumerate(cfg.get("models", [])):
            gen = {"icosphere": M.icosphere, "wavy_icosphere": M.wavy_icosphere}[m["kind"]]
            r.set_model(k, *gen(m["level"]))
        tris, depth = r.model_info()
        r.render(1, spp)  # JIT compile + BVH build + scratch planes + first touch
        r.clear()
        kms = []
        t0 = time.perf_counter()
        for s in range(args.steps):
            r.render(1 + s * spp, spp)
            kms.append(r.last_kernel_ms()[0])
        dt = time.perf_counter() - t0
        samples = w * h * spp * args.steps
        print(json.dumps({"config": key, "name": name, "width": w, "height": h, "spp_per_step": spp,
                          "steps": args.steps, "Msamples_s": round(samples / dt / 1e6, 2),
                          "kernel_Msamples_s": round(w * h * spp / (sum(kms) / len(kms) / 1e3) / 1e6, 2),
                          "kernel_ms_per_step": round(sum(kms) / len(kms), 3), "triangles": tris,
                          "bvh_depth": depth, "overrides": over}), flush=True)
        r.close()


if __name__ == "__main__":
    main()
