#!/usr/bin/env python3
"""C5 at 1024^2, 4 passes: the 81,920-triangle icosphere through the LBVH vs
the same scene with an analytic SPHERE in its place -- the BVH's share."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "raytracer-0_amd"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402  (configs.json loader only)
import rt0  # noqa: E402
from rt0 import meshes as M  # noqa: E402


def run(cfg, cfgs, models, n=1024, spp=4):
    r = rt0.Renderer(n, n)
    rt0.configure(r, cfg, cfgs)
    for k, m in enumerate(models):
        r.set_model(k, *M.icosphere(m["level"]))
    r.render(1, spp)
    ms = []
    for s in range(3):
        r.render(1 + spp * (s + 1), spp)
        ms.append(r.last_kernel_ms()[0])
    r.close()
    return sum(ms) / len(ms)


def main():
    cfgs = O.load_configs()
    cfg = dict([c for c in cfgs["configs"] if c["name"] == "c5_spectral_models"][0])
    t_bvh = run(cfg, cfgs, cfg["models"])
    sph = dict(cfg)
    sph["scene_lines"] = [l.replace("TRIANGLE", "SPHERE") for l in cfg["scene_lines"]]
    t_sph = run(sph, cfgs, [])
    print(json.dumps({"bvh_ms": round(t_bvh, 3), "sphere_ms": round(t_sph, 3)}))


if __name__ == "__main__":
    main()
