#!/usr/bin/env python3
"""Steady-state kernel time of the pass kernel from a rocprofv3 --kernel-trace
run of bench.py (scripts/gpu_measure.sh).

    [HALVES=K] kt_summary.py OUT.json TRACE_DIR SKIP

Keeps the rt0_jit_pass dispatches after the first SKIP (the warm-up step's
launches) and reports their median / mean / min / max duration, plus the other
kernels' totals (rocprofv3's own --stats table averages every dispatch,
warm-up included).  A deferred ReSTIR pass is two or three dispatches (rt0_jit_pass,
rt0_jit_nee [, rt0_jit_resolve]; rt0_integrator.h RT0_FUSED_RESOLVE), four in scenes with models
(+ rt0_jit_walk), twice when the pass runs as two row parts on K streams
(restir_split_pass): "median_ms" .. "max_ms" are then per pass, each pass's
span (first dispatch start to last end), and the per-kernel medians its busy
time per pass.
Wavefront launches (rt0_jit_wf_*: shade, plan and march or walk per round)
are summed launch by launch with what completes them: rt0_sum_kernel, or a
ReSTIR pass's nee (+ walk) + resolve.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

KERNEL = "rt0_jit_pass"
GROUP = ("rt0_jit_pass", "rt0_jit_nee", "rt0_jit_walk", "rt0_jit_resolve", "rt0_jit_wf_shade", "rt0_jit_wf_plan",
         "rt0_jit_wf_march", "rt0_jit_wf_walk")
# a wavefront SDF launch (rt0_integrator.h wf_shade_body): MAX_BOUNCES + 2
# shade and MAX_BOUNCES + 1 march dispatches, then one rt0_sum_kernel; a
# wavefront ReSTIR pass: MAX_BOUNCES + 1 shade and MAX_BOUNCES walk
# dispatches, then rt0_jit_nee (+ rt0_jit_walk) + rt0_jit_resolve
WF = ("rt0_jit_wf_shade", "rt0_jit_wf_plan", "rt0_jit_wf_march", "rt0_jit_wf_walk")
TAIL = ("rt0_jit_nee", "rt0_jit_walk", "rt0_jit_resolve")


def main():
    out, d, skip = sys.argv[1], sys.argv[2], int(sys.argv[3])
    halves = int(os.environ.get("HALVES", "1"))
    rows = []
    for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(fn)))
    rows.sort(key=lambda r: float(r["Start_Timestamp"]))
    dur = {k: [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].strip() == k]
           for k in GROUP}
    pas = dur[KERNEL]
    per_kernel = {}
    sums = [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in rows
            if r["Kernel_Name"].strip().startswith("rt0_sum_kernel")]
    wf = bool(dur["rt0_jit_wf_march"] or dur["rt0_jit_wf_walk"])
    if wf and (sums or dur["rt0_jit_resolve"]):  # wavefront launches: every dispatch of the launch + its tail, per launch
        tail = {k: dur[k] for k in TAIL if dur[k]} if dur["rt0_jit_resolve"] else {"rt0_sum_kernel": sums}
        nl = min(len(v) for v in tail.values())
        per = {k: len(dur[k]) // nl for k in WF if dur[k]}
        # a launch's time is its span: from its first dispatch's start to the
        # end of the dispatch that completes it (rt0_sum_kernel, or resolve) --
        # the halves on two HIP streams overlap, so the kernels' durations
        # summed would count the overlap twice (kept as per-kernel busy time)
        last = "rt0_jit_resolve" if dur["rt0_jit_resolve"] else None
        ends = [float(r["End_Timestamp"]) for r in rows
                if (r["Kernel_Name"].strip() == last if last else r["Kernel_Name"].strip().startswith("rt0_sum_kernel"))]
        mine = set(GROUP)
        starts = sorted(float(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].strip() in mine)
        pas, lo = [], 0
        for i in range(nl):
            first = [t for t in starts[lo:] if t < ends[i]]
            pas.append(ends[i] - first[0] if first else 0.0)
            lo += len(first)
        per_kernel = {k: statistics.median([sum(dur[k][i * per[k]:(i + 1) * per[k]]) for i in range(skip, nl)]) / 1e6
                      for k in per if nl > skip}
        per_kernel.update({k: statistics.median(v[skip:nl]) / 1e6 for k, v in tail.items() if nl > skip})
        per_kernel["dispatches_per_launch"] = per
    elif dur["rt0_jit_nee"]:  # deferred passes: pass + nee (+ walk) + resolve per pass, or per half
        # A pass is one rt0_jit_pass dispatch, or two when it runs as two row
        # halves on two streams (rt0_host.cpp restir_split_pass; they
        # overlap): env HALVES = K (scripts/gpu_measure.sh sets it); a pass's
        # time is its span, first start to last end; per kernel: its busy
        # time per pass (halves summed)
        groups, seen = [], 0
        for r in rows:
            name = r["Kernel_Name"].strip()
            if name not in GROUP:
                continue
            if name == KERNEL:
                if seen % halves == 0:
                    groups.append([])
                seen += 1
            if groups:
                groups[-1].append((name, float(r["Start_Timestamp"]), float(r["End_Timestamp"])))
        pas = [max(g[2] for g in gr) - min(g[1] for g in gr) for gr in groups]
        per_kernel = {k: statistics.median([sum(g[2] - g[1] for g in gr if g[0] == k) for gr in groups[skip:]]) / 1e6
                      for k in GROUP if dur[k] and groups[skip:]}
        per_kernel["dispatches_per_pass"] = {k: sum(1 for g in groups[-1] if g[0] == k) for k in GROUP if dur[k]}
    kept = pas[skip:]
    other = defaultdict(list)
    for r in rows:
        if r["Kernel_Name"].strip() not in GROUP and not (wf and r["Kernel_Name"].startswith("rt0_sum_kernel")):
            other[r["Kernel_Name"][:80]].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    res = {"kernel": "+".join(k for k in GROUP if dur[k]) if wf else KERNEL, "dispatches": len(pas), "skipped": skip, "kept": len(kept),
           "median_ms": statistics.median(kept) / 1e6 if kept else None,
           "mean_ms": statistics.mean(kept) / 1e6 if kept else None,
           "min_ms": min(kept) / 1e6 if kept else None, "max_ms": max(kept) / 1e6 if kept else None,
           "per_kernel_median_ms": per_kernel,
           "all_ms": [round(x / 1e6, 4) for x in pas],
           "other_kernels": {k: {"calls": len(v), "total_ms": sum(v) / 1e6} for k, v in other.items()}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("all_ms", "other_kernels")}))


if __name__ == "__main__":
    main()
