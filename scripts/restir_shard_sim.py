"""Load balance of the ReSTIR row sharding on one device: each
rank's share of a pass rendered alone (rt0_set_shard on one renderer, after
warm-up passes of the whole image), for contiguous blocks (block_band) and
for two round-robin bands per rank (interleaved_band, the bench's split), on
the C3 and C5 bench workloads.  Prints per-rank pass times and the strong-
scaling ceiling T1 / (N * slowest rank) (halo exchange and gather excluded)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
import rt0.shard as shard  # noqa: E402
from rt0 import workloads  # noqa: E402

out = {}
for key in sys.argv[1:] or ["c3", "c5"]:
    wl = workloads.get(key)
    W, H = wl["width"], wl["height"]
    r = rt0.Renderer(W, H)
    workloads.configure(r, wl)
    r.render(1, 4)  # reservoirs warm (temporal reuse starts at pass 3)
    state = {"frame": 5}

    def timed():
        ts = []
        for _ in range(3):
            r.render(state["frame"], 1)
            state["frame"] += 1
            ts.append(r.last_kernel_ms()[0])
        return min(ts)

    t1 = timed()
    res = {"whole_ms": round(t1, 3)}
    r.set_halo(24)
    for n in (2, 4, 8):
        for split, band in (("contiguous", shard.block_band(H, n)), ("round_robin", shard.interleaved_band(H, n))):
            per_rank = []
            for rank in range(n):
                r.set_shard(rank, n, band)
                per_rank.append(timed())
            r.set_shard(0, 1, 16)
            mean = sum(per_rank) / n
            res["%d_%s" % (n, split)] = {"band": band, "rank_ms": [round(t, 3) for t in per_rank],
                                         "max_over_mean": round(max(per_rank) / mean, 3),
                                         "ceiling": round(t1 / (n * max(per_rank)), 3)}
            print(key, n, split, res["%d_%s" % (n, split)], flush=True)
    r.close()
    out[key] = res
print(json.dumps(out))
