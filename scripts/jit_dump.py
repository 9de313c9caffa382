#!/usr/bin/env python3
"""Compile the scene-specialised kernel of one configs.json entry offline
(hipRTC, no GPU needed) and keep its source and code object for inspection:

    RT0_JIT_DUMP=/tmp/jd/c2 python scripts/jit_dump.py c2_cornell_mis_8
    llvm-readelf --notes /tmp/jd/c2_*.co      # VGPRs, SGPRs, scratch, LDS
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "raytracer-0_amd"), os.path.join(REPO, "oracle")]

import oracle as O  # noqa: E402  (configs.json loader only)
import rt0  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2_cornell_mis_8"
    cfgs = O.load_configs()
    cfg = [c for c in cfgs["configs"] if c["name"] == name][0]
    c = rt0.parse_config(*rt0.config_strings(cfg))
    scene, sdf = rt0.scene_strings(cfg, cfgs)
    print(name, "code object bytes:", rt0.jit_compile(scene, sdf, c))


if __name__ == "__main__":
    main()
