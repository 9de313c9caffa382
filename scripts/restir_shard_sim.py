"""Load balance of the ReSTIR row-block sharding on one device:
each of the N row blocks (RestirShard's split: ceil(H/N) rows rounded to 16)
rendered alone through the viewport, after warm-up passes of the whole image,
for the C3 and C5 bench workloads.  Prints per-block pass times and the
strong-scaling ceiling T1 / (N * max block) that the slowest block allows
(halo exchange and gather excluded)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "raytracer-0_amd"))
import rt0  # noqa: E402
from rt0 import workloads  # noqa: E402

out = {}
for key in sys.argv[1:] or ["c3", "c5"]:
    wl = workloads.get(key)
    W, H = wl["width"], wl["height"]
    r = rt0.Renderer(W, H)
    workloads.configure(r, wl)
    r.render(1, 4)  # reservoirs warm (temporal reuse starts at pass 3)
    frame = 5

    def timed(y0, rows):
        global frame
        r.set_viewport(0, y0, W, rows)
        ts = []
        for _ in range(3):
            r.render(frame, 1)
            frame += 1
            ts.append(r.last_kernel_ms()[0])
        return min(ts)

    t1 = timed(0, H)
    res = {"whole_ms": round(t1, 3)}
    for n in (2, 4, 8):
        band = -(-H // n)
        band = -(-band // 16) * 16
        blocks = [timed(y0, min(band, H - y0)) for y0 in range(0, H, band)]
        res[n] = {"block_ms": [round(b, 3) for b in blocks], "max_over_mean": round(max(blocks) / (sum(blocks) / len(blocks)), 3),
                  "ceiling": round(t1 / (n * max(blocks)), 3)}
        print(key, n, res[n], flush=True)
    r.set_viewport(0, 0, 0, 0)
    r.close()
    out[key] = res
print(json.dumps(out))
