"""Load balance of the progressive workloads' 16-row round-robin band sharding
(bench.py Progressive, rt0_set_shard) on one device: every rank's share of
one bench step rendered alone (the other ranks' bands skipped), for N = 2, 4,
8, under strong scaling (spp passes split N ways) and under bench.py's
default weak scaling (N x spp passes, each rank its rows for all of them).  Prints per-rank kernel times (HIP events, best of 3), max/mean, the
strong-scaling ceiling T1 / (N * slowest rank) and the sum of the ranks'
times over T1 (how much per-rank overhead sharding adds) -- the gather and
RCCL are excluded.

    python3 scripts/shard_sim.py c4 [c2 ...] > profiles/rNN/shard_sim/shard_sim.txt

ReSTIR workloads (C3, C5: one pass per call, reservoir halo rows exchanged
between passes -- here each rank renders alone, without the exchange) are
simulated per pass for the partitions rt0.shard offers: one contiguous block
per rank, and `per_rank` round-robin bands per rank (interleaved_band), for
per_rank = 2, 4, 8 (band >= 2 x halo).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

BAND = 16


def restir_sim(key, wl):
    from rt0 import shard
    W, H = wl["width"], wl["height"]
    halo = 24

    def timed(rank=0, n=1, band=None, rows=None):
        r = rt0.Renderer(W, H)
        workloads.configure(r, wl)
        if rows is not None:  # a contiguous row block as a viewport rectangle
            r.set_viewport(0, rows[0], W, rows[1] - rows[0])
        elif n > 1:
            r.set_shard(rank, n, band)
            r.set_halo(halo)
        ts = []
        for k in range(1, 6):  # one pass per call; the first two warm up
            r.render(k, 1)
            if k > 2:
                ts.append(r.last_kernel_ms()[0])
        path = r.last_render_path()
        r.close()
        return min(ts), path

    t1, path = timed()
    res = {"whole_ms": round(t1, 3), "render_path": path, "halo": halo}
    print(key, "whole", res, flush=True)
    # per-row-band cost (64 bands), for contiguous blocks cut at equal cost
    nb = 64
    bh = H // nb
    cost = [timed(rows=(b * bh, (b + 1) * bh))[0] for b in range(nb)]
    res["band_ms"] = [round(c, 4) for c in cost]
    print(key, "band costs", res["band_ms"], flush=True)
    for n in (2, 4, 8):
        cuts = shard.cost_cuts(cost, bh, H, n)
        per = [timed(rows=(cuts[k], cuts[k + 1]))[0] for k in range(n)]
        mean = sum(per) / n
        res["%d_contiguous_cost" % n] = d = {"cuts": cuts, "rank_ms": [round(t, 3) for t in per],
                                              "max_over_mean": round(max(per) / mean, 3),
                                              "ceiling": round(t1 / (n * max(per)), 3),
                                              "sum_over_whole": round(sum(per) / t1, 3)}
        print(key, n, "contiguous_cost", d, flush=True)
    for n in (2, 4, 8):
        parts = [("contiguous", shard.block_band(H, n))]
        for per in (2, 4, 8):
            b = shard.interleaved_band(H, n, per_rank=per, halo=halo)
            if b * n < H:
                parts.append(("round_robin_%d" % per, b))
        for name, band in parts:
            per = [timed(rank, n, band)[0] for rank in range(n)]
            mean = sum(per) / n
            res["%d_%s" % (n, name)] = d = {"band": band, "rank_ms": [round(t, 3) for t in per],
                                            "max_over_mean": round(max(per) / mean, 3),
                                            "ceiling": round(t1 / (n * max(per)), 3),
                                            "sum_over_whole": round(sum(per) / t1, 3)}
            print(key, n, name, d, flush=True)
    return res


def main():
    out = {}
    for key in sys.argv[1:] or ["c4"]:
        wl = workloads.get(key)
        if workloads.restir(wl):
            out[key] = restir_sim(key, wl)
            continue
        W, H, spp = wl["width"], wl["height"], wl["spp"]

        def timed(rank, n, frames=None):
            frames = frames or spp
            r = rt0.Renderer(W, H)
            workloads.configure(r, wl)
            if n > 1:
                r.set_shard(rank, n, BAND)
            r.render(1, frames)  # warm-up (JIT compile, buffers)
            ts = []
            for k in range(3):
                r.clear()
                r.render(1 + frames * (k + 1), frames)
                ts.append(r.last_kernel_ms()[0])
            path = r.last_render_path()
            r.close()
            return min(ts), path

        t1, path = timed(0, 1)
        res = {"whole_ms": round(t1, 3), "render_path": path, "band_rows": BAND, "spp": spp}
        print(key, "whole", res, flush=True)
        for n in (2, 4, 8):
            per = [timed(rank, n)[0] for rank in range(n)]
            mean = sum(per) / n
            res[str(n)] = {"rank_ms": [round(t, 3) for t in per], "max_over_mean": round(max(per) / mean, 3),
                           "ceiling": round(t1 / (n * max(per)), 3), "sum_over_whole": round(sum(per) / t1, 3)}
            print(key, n, res[str(n)], flush=True)
            # bench.py's default N > 1 step (weak scaling): n x spp passes, each
            # rank its 1/n of the rows for all of them -- the ceiling is the N = 1
            # step time over the slowest rank's
            perw = [timed(rank, n, spp * n)[0] for rank in range(n)]
            res[str(n) + "_weak"] = {"rank_ms": [round(t, 3) for t in perw],
                                     "max_over_mean": round(max(perw) * n / sum(perw), 3),
                                     "ceiling": round(t1 / max(perw), 3)}
            print(key, n, "weak", res[str(n) + "_weak"], flush=True)
        out[key] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
