#!/usr/bin/env python3
"""Steady-state kernel time of the pass kernel from a rocprofv3 --kernel-trace
run of bench.py (scripts/gpu_measure.sh).

    kt_summary.py OUT.json TRACE_DIR SKIP

Keeps the rt0_jit_pass dispatches after the first SKIP (the warm-up step's
launches) and reports their median / mean / min / max duration, plus the other
kernels' totals (rocprofv3's own --stats table averages every dispatch,
warm-up included).
"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict

KERNEL = "rt0_jit_pass"


def main():
    out, d, skip = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(fn)))
    rows.sort(key=lambda r: float(r["Start_Timestamp"]))
    pas = [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in rows if KERNEL in r["Kernel_Name"]]
    kept = pas[skip:]
    other = defaultdict(list)
    for r in rows:
        if KERNEL not in r["Kernel_Name"]:
            other[r["Kernel_Name"][:80]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    res = {"kernel": KERNEL, "dispatches": len(pas), "skipped": skip, "kept": len(kept),
           "median_ms": statistics.median(kept) / 1e6 if kept else None,
           "mean_ms": statistics.mean(kept) / 1e6 if kept else None,
           "min_ms": min(kept) / 1e6 if kept else None, "max_ms": max(kept) / 1e6 if kept else None,
           "all_ms": [round(x / 1e6, 4) for x in pas],
           "other_kernels": {k: {"calls": len(v), "total_ms": sum(v) / 1e6} for k, v in other.items()}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("all_ms", "other_kernels")}))


if __name__ == "__main__":
    main()
