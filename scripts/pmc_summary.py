#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of one workload (scripts/gpu_measure.sh)
into per-launch figures of the scene-specialised pass kernel (rt0_jit_pass).

    pmc_summary.py OUT.json W H BYTES_PER_PIXEL SKIP PASS_DIR [PASS_DIR ...]

Per dispatch of rt0_jit_pass (the counting instance bench.py launches
afterwards is a different kernel and is excluded), dropping the first SKIP
dispatches (the warm-up step), averaged over the rest -- for a deferred ReSTIR
pass (rt0_jit_pass + rt0_jit_nee [+ rt0_jit_walk] + rt0_jit_resolve, each
once per pass or, split into K row parts, twice) the kernels' dispatches
summed per pass:
  * HBM traffic: FETCH_SIZE x 2 (MI355X_MICROARCH.md: gfx950 reports half the
    bytes of a 16-B/lane streaming read; scripts/fetch_calib.hip measures the
    factor for the 64-B gathers and bilinear taps of the ReSTIR/BVH kernels)
    + WRITE_SIZE (exact for 16-B/lane stores); counters in KiB;
  * VALU: SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32, SQ_ACTIVE_INST_VALU,
    SQ_THREAD_CYCLES_VALU -> lane utilisation (active lanes per issued VALU
    instruction / 64);
  * clock: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / dispatch duration
    = the effective shader clock under load (DVFS give-back);
  * stall split: SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as shares of
    SQ_WAVE_CYCLES.
The algorithmic bytes per launch = W x H x BYTES_PER_PIXEL (32: one float4
accumulator read + write; 160 for a ReSTIR pass: + two reservoir MRT writes
and the six reservoir planes read once).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "rt0_jit_pass"
GROUP = ("rt0_jit_pass", "rt0_jit_nee", "rt0_jit_walk", "rt0_jit_resolve", "rt0_jit_wf_shade", "rt0_jit_wf_plan", "rt0_jit_wf_march")
# wavefront SDF launches (rt0_integrator.h wf_shade_body): MAX_BOUNCES + 2
# shade and MAX_BOUNCES + 1 march dispatches per launch, closed by one
# rt0_sum_kernel -- their counters are summed per launch
WF = ("rt0_jit_wf_shade", "rt0_jit_wf_plan", "rt0_jit_wf_march")


def launches_in(d):
    """rt0_sum_kernel dispatches of a pass directory: one per wavefront launch."""
    ids = set()
    for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Kernel_Name"].strip().startswith("rt0_sum_kernel"):
                ids.add(int(r["Dispatch_Id"]))
    return len(ids)


def dispatches(d, kernel):
    """{dispatch id: {counter: value}} and {dispatch id: duration ns} of one
    kernel in one pass directory."""
    vals = defaultdict(lambda: defaultdict(float))
    for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Kernel_Name"].strip() == kernel:
                vals[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Kernel_Name"].strip() == kernel:
                dur[int(r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return vals, dur


def main():
    out, W, H, bpp, skip = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5])
    per = {}  # counter -> mean over the kept dispatches
    n_kept = {}
    clock = []
    kernels = []
    by_kernel = {}  # kernel -> {counter: mean per dispatch}
    for d in sys.argv[6:]:
        in_dir = {}  # this pass directory's counters, the group's kernels summed
        nl = launches_in(d)
        for kernel in GROUP:
            vals, dur = dispatches(d, kernel)
            every = sorted(vals)
            per_launch = 1
            if kernel in WF and nl > skip:
                per_launch = max(1, len(every) // nl)
            elif kernel not in WF:
                # env HALVES = K: ReSTIR passes split into K row parts
                # (rt0_host.cpp restir_split_pass) dispatch each kernel twice
                per_launch = int(os.environ.get("HALVES", "1"))
            ids = every[skip * per_launch:]
            if not ids:
                continue
            if kernel not in kernels:
                kernels.append(kernel)
            names = set().union(*(vals[i].keys() for i in ids))
            for c in names:  # per pass: the group's kernels summed (a wavefront launch's dispatches summed)
                m = sum(vals[i].get(c, 0.0) for i in ids) / len(ids) * per_launch
                in_dir[c] = in_dir.get(c, 0.0) + m
                by_kernel.setdefault(kernel, {})[c] = m
                n_kept[c] = len(ids)
            if "GRBM_GUI_ACTIVE" in names and kernel in (KERNEL, "rt0_jit_wf_march"):
                for i in ids:
                    if dur.get(i):
                        clock.append(vals[i]["GRBM_GUI_ACTIVE"] / 8.0 / dur[i])  # cycles per ns = GHz
        per.update(in_dir)  # a counter collected in two passes: the later pass's value
    res = {"kernel": "+".join(kernels) or KERNEL, "skipped_dispatches": skip, "dispatches_kept": n_kept, "counters": per,
           "algorithmic_bytes_per_launch": W * H * bpp}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        res["fetch_bytes_per_launch"] = 2.0 * per["FETCH_SIZE"] * 1024.0
        res["write_bytes_per_launch"] = per["WRITE_SIZE"] * 1024.0
        res["traffic_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
        res["note"] = "FETCH_SIZE x2 (gfx950 16-B/lane read correction), WRITE_SIZE as reported; KiB -> bytes"
    if "SQ_THREAD_CYCLES_VALU" in per:
        res["valu"] = {c: per[c] for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_ACTIVE_INST_VALU",
                                           "SQ_THREAD_CYCLES_VALU") if c in per}
        res["valu_lane_utilisation"] = per["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64.0 * per["SQ_ACTIVE_INST_VALU"])
    if len(by_kernel) > 1:
        res["per_kernel"] = by_kernel
        res["per_kernel_lane_utilisation"] = {
            k: v["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64.0 * v["SQ_ACTIVE_INST_VALU"])
            for k, v in by_kernel.items() if "SQ_THREAD_CYCLES_VALU" in v and "SQ_ACTIVE_INST_VALU" in v}
    if clock:
        clock.sort()
        res["clock_ghz_median"] = clock[len(clock) // 2]
    if "SQ_WAVE_CYCLES" in per:
        w = per["SQ_WAVE_CYCLES"] or 1.0
        res["stall_share"] = {c: per[c] / w for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_BUSY_CYCLES")
                              if c in per}
    if "SQ_INSTS_VALU_FMA_F32" in per:
        tot = per.get("SQ_INSTS_VALU") or 1.0
        res["valu_mix"] = {c[len("SQ_INSTS_VALU_"):].lower(): per[c] / tot for c in per
                           if c.startswith("SQ_INSTS_VALU_")}
        # wave-level FP32 operations the hardware executed (FMA = 2): the
        # ceiling the algorithmic FLOP model is compared against
        res["hw_flop_wave_instr"] = 2.0 * per["SQ_INSTS_VALU_FMA_F32"] + per["SQ_INSTS_VALU_ADD_F32"] + \
            per["SQ_INSTS_VALU_MUL_F32"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("counters", "per_kernel")}))


if __name__ == "__main__":
    main()
