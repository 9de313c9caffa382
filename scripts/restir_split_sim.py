"""Row parts per ReSTIR pass (RT0_RESTIR_SPLIT) against the shard size: one
rank's share of a pass rendered alone on one device (its round-robin bands
of rt0_set_shard, halo set, no exchange -- as scripts/shard_sim.py), for the
bench's N > 1 partition (bench.py Restir: four bands per rank where each stays
>= 64 rows, else two), under each split setting.  Prints per-rank kernel
times (HIP events, best of 3 passes after 2 warm-up passes), the slowest rank
and the strong-scaling ceiling T1 / (N * slowest).

    python3 scripts/restir_split_sim.py c5 [N ...] > profiles/rNN/.../split_sim.txt
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import shard, workloads  # noqa: E402

SPLITS = tuple(os.environ.get("SPLITS", "0 2 3 4").split())  # e.g. SPLITS=0 RT0_DEFER_NEE=0


def timed(wl, rank=0, n=1, band=None, halo=24):
    r = rt0.Renderer(wl["width"], wl["height"])
    workloads.configure(r, wl)
    if n > 1:
        r.set_shard(rank, n, band)
        r.set_halo(halo)
    ts = []
    for k in range(1, 6):  # one pass per call; the first two warm up
        r.render(k, 1)
        if k > 2:
            ts.append(r.last_kernel_ms()[0])
    r.close()
    return min(ts)


def main():
    key = sys.argv[1] if len(sys.argv) > 1 else "c5"
    ns = [int(a) for a in sys.argv[2:]] or [2, 4, 8]
    wl = workloads.get(key)
    H = wl["height"]
    out = {}
    for sp in SPLITS:
        os.environ["RT0_RESTIR_SPLIT"] = sp  # read per render (rt0_host.cpp restir_split_parts)
        t1 = timed(wl)
        res = {"whole_ms": round(t1, 3)}
        print(key, "split", sp, "whole", res["whole_ms"], flush=True)
        for n in ns:
            per = 4 if H >= n * 4 * 64 else 2
            band = shard.interleaved_band(H, n, per_rank=per)
            ms = [timed(wl, rank, n, band) for rank in range(n)]
            d = {"band": band, "rank_ms": [round(t, 3) for t in ms], "slowest_ms": round(max(ms), 3),
                 "ceiling": round(t1 / (n * max(ms)), 3), "sum_over_whole": round(sum(ms) / t1, 3)}
            res[str(n)] = d
            print(key, "split", sp, "N", n, d, flush=True)
        out[sp] = res
    print(json.dumps({key: out}))


if __name__ == "__main__":
    main()
