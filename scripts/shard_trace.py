"""One rank's share of a bench step, rendered alone (rank R of N, 16-row
round-robin bands; ReSTIR workloads: BAND-row bands, one pass per call), for
a kernel trace of a sharded launch:
    rocprofv3 --kernel-trace ... -- python3 scripts/shard_trace.py c4 0 8 [BAND]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

key, rank, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
wl = workloads.get(key)
r = rt0.Renderer(wl["width"], wl["height"])
workloads.configure(r, wl)
if workloads.restir(wl):
    if n > 1:
        r.set_shard(rank, n, int(sys.argv[4]) if len(sys.argv) > 4 else 64)
        r.set_halo(24)
    for k in range(1, 7):
        r.render(k, 1)
        print("pass", k, r.last_kernel_ms(), r.last_render_path(), flush=True)
    sys.exit(0)
if n > 1:
    r.set_shard(rank, n, 16)
for k in range(3):
    r.clear()
    r.render(1 + wl["spp"] * k, wl["spp"])
    print("launch", k, r.last_kernel_ms(), r.last_render_path(), flush=True)
