#!/usr/bin/env python3
"""Write the C5 model's world-space triangles (rt0/workloads.json c5, as
librt0's build instances them), build scripts/bvh_quality.cpp against
rt0_bvh_sah.cpp and run it: nodes visited per ray, device-LBVH shape vs the
binned-SAH tree, on C5-like ray sets (CPU only).

    python3 scripts/bvh_quality.py [workload]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "raytracer-0_amd"))

import numpy as np  # noqa: E402

from rt0 import meshes, workloads  # noqa: E402


def main():
    wl = workloads.get(sys.argv[1] if len(sys.argv) > 1 else "c5")
    soup = [meshes.world_triangles(v, t, pos, scale) for v, t, pos, scale, _ in workloads.model_instances(wl)]
    tri = "/tmp/rt0_bvhq_tris.f32"
    np.concatenate(soup).astype(np.float32).tofile(tri)
    exe = "/tmp/rt0_bvhq"
    csrc = os.path.join(REPO, "raytracer-0_amd", "csrc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-include",
                           "functional", os.path.join(HERE, "bvh_quality.cpp"), os.path.join(csrc, "rt0_bvh_sah.cpp"),
                           "-o", exe, "-lpthread"])
    subprocess.check_call([exe, tri])


if __name__ == "__main__":
    main()
