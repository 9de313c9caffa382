"""Per-GPU kernel time of one shard (rank 0 of N) on one device: the strong-
scaling ceiling of the band sharding without any collective."""
import json, os, sys, time
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd")); sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import rt0, oracle as O
cfgs = O.load_configs()
cfg = [c for c in cfgs["configs"] if c["name"] == "c2_cornell_mis_8"][0]
res = {}
for n in (1, 2, 4, 8):
    r = rt0.Renderer(1024, 1024)
    rt0.configure(r, cfg, cfgs)
    r.set_shard(0, n, 16)
    r.render(1, 64)
    ts = []
    for _ in range(5):
        r.clear(); r.render(1, 64); ts.append(r.last_kernel_ms()[0])
    res[n] = min(ts)
    print(n, "shard kernel ms", res[n], "ideal", res[1] / n, "efficiency %.3f" % (res[1] / n / res[n]), flush=True)
