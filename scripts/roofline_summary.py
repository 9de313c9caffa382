"""Per-workload roofline table from a profile directory written by
scripts/gpu_round2.sh (bench_<c>.json, kernel_stats_<c>.csv from
rocprofv3 --kernel-trace --stats, pmc_<c>.json from scripts/pmc_traffic.py).

frac is recomputed from the rocprof average duration of the scene-specialised
pass kernel (rt0_jit_pass), not from bench.py's live HIP-event time:
  achieved = FLOP/sample (bench.py's model x counted events) x samples per
             launch / rocprof average launch duration
VALU issue utilisation = (SQ_INSTS_VALU x 2 + SQ_INSTS_VALU_TRANS_F32 x 2) SIMD
cycles / (1024 SIMDs x launch duration x 2.4 GHz) (wave64 VALU = 2 passes on a
SIMD32-wide datapath; transcendentals quarter rate -> 4 cycles).
usage: python scripts/roofline_summary.py profiles/r02/s2 > profiles/r02/s2/roofline.md
"""
import csv
import json
import os
import sys

PEAK = 157.3
D = sys.argv[1]
rows = []
for c in ("c1", "c2", "c3", "c4", "c5"):
    try:
        b = json.load(open(os.path.join(D, "bench_%s.json" % c)))
    except FileNotFoundError:
        continue
    ks = {}
    with open(os.path.join(D, "kernel_stats_%s.csv" % c)) as f:
        for r in csv.DictReader(f):
            ks[r["Name"]] = r
    k = ks.get("rt0_jit_pass")
    avg_ns = float(k["AverageNs"]) if k else float("nan")
    cfg = b["config"]
    # pass-kernel launches per step: the profiled command runs 1 warm-up + 2
    # steps (scripts/gpu_round2.sh); a frame-chunked launch adds a sum kernel
    # that is not a pass
    per_step = int(k["Calls"]) / 3.0 if k else b["roofline"]["launches_per_step"]
    spl = cfg["width"] * cfg["height"] * cfg["spp"] / per_step
    fps = b["roofline"]["flop_per_sample"]
    ach = fps * spl / (avg_ns * 1e-9) / 1e12
    pmc = {}
    try:
        pmc = json.load(open(os.path.join(D, "pmc_%s.json" % c)))
    except FileNotFoundError:
        pass
    v = pmc.get("valu", {})
    issue = float("nan")
    if v:
        cyc = 2.0 * (v["SQ_INSTS_VALU"] - v["SQ_INSTS_VALU_TRANS_F32"]) + 4.0 * v["SQ_INSTS_VALU_TRANS_F32"]
        issue = cyc / (1024 * avg_ns * 1e-9 * 2.4e9)  # counters are per dispatch (pmc_traffic.py)
    rows.append(dict(config=c, workload=cfg["workload"], msamples_s=b["value"], flop_per_sample=fps,
                     samples_per_launch=spl, rocprof_avg_ms=avg_ns / 1e6, achieved_tflops=ach, frac=ach / PEAK,
                     bench_frac=b["roofline"]["frac"], lane_util=pmc.get("valu_lane_utilisation"),
                     valu_issue_util=issue, traffic_bytes=pmc.get("traffic_bytes_per_launch"),
                     algorithmic_bytes=pmc.get("algorithmic_bytes_per_launch"),
                     events=b["roofline"].get("events_per_sample")))
json.dump(rows, open(os.path.join(D, "roofline.json"), "w"), indent=1)
print("| config | Msamples/s | FLOP/sample | rocprof ms/launch | TFLOP/s | frac (rocprof) | frac (bench) | "
      "VALU lane util | VALU issue util | HBM bytes/launch (PMC / algorithmic) |")
print("|---|---|---|---|---|---|---|---|---|---|")
for r in rows:
    print("| %s | %.0f | %.0f | %.3f | %.1f | %.3f | %.3f | %s | %s | %s / %s |" % (
        r["config"], r["msamples_s"], r["flop_per_sample"], r["rocprof_avg_ms"], r["achieved_tflops"], r["frac"],
        r["bench_frac"], "%.2f" % r["lane_util"] if r["lane_util"] else "-",
        "%.2f" % r["valu_issue_util"] if r["valu_issue_util"] == r["valu_issue_util"] else "-",
        "%.3g" % r["traffic_bytes"] if r["traffic_bytes"] else "-",
        "%.3g" % r["algorithmic_bytes"] if r["algorithmic_bytes"] else "-"))
