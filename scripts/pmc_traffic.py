#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_pmc.sh)
into per-launch HBM traffic of the integrator kernel.

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports half
the bytes of a 16-B-per-lane streaming read -- doubled here; WRITE_SIZE is exact
for 16-B-per-lane stores.  Both counters are in KiB.

usage: pmc_traffic.py <fetch pass dir> <write pass dir> <out.json> [W H [valu pass dir [bytes/pixel]]]

bytes/pixel = algorithmic HBM bytes per pixel per launch: 32 for the
progressive kernel (one float4 accumulator read + write), 160 for a ReSTIR
pass (+ two reservoir MRT writes and the six reservoir input planes read once).
"""
import csv
import json
import sys
from collections import defaultdict

KERNELS = ("rt0_jit_pass", "rt0_pass_kernel")


def per_dispatch(path, counter):
    """Counter per dispatch of the timed kernel: the JIT kernel when the run used
    it (the counting instance bench.py launches afterwards is excluded)."""
    rows = [r for r in csv.DictReader(open(path + "/run_counter_collection.csv")) if r["Counter_Name"] == counter]
    kern = next((k for k in KERNELS if any(k in r["Kernel_Name"] for r in rows)), KERNELS[0])
    acc = defaultdict(float)
    name = {}
    for r in rows:
        if kern not in r["Kernel_Name"]:
            continue
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"]
    return acc, name


def main():
    fdir, wdir, out = sys.argv[1:4]
    W, H = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (1024, 1024)
    f, fn = per_dispatch(fdir, "FETCH_SIZE")
    w, wn = per_dispatch(wdir, "WRITE_SIZE")
    fetch = [2.0 * v * 1024.0 for v in f.values()]  # KiB -> B, x2 gfx950 read correction
    write = [v * 1024.0 for v in w.values()]
    res = {
        "kernel": sorted(set(fn.values()) | set(wn.values())),
        "dispatches": [len(fetch), len(write)],
        "fetch_bytes_per_launch": sum(fetch) / max(1, len(fetch)),
        "write_bytes_per_launch": sum(write) / max(1, len(write)),
        "algorithmic_bytes_per_launch": W * H * (float(sys.argv[7]) if len(sys.argv) > 7 else 32.0),
        "note": "FETCH_SIZE x2 (gfx950 16-B/lane read correction), WRITE_SIZE as reported; KiB -> bytes",
    }
    res["traffic_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
    if len(sys.argv) > 6 and sys.argv[6] != "-":  # optional VALU pass: SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
        v = {}
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU"):
            d, _ = per_dispatch(sys.argv[6], c)
            v[c] = sum(d.values()) / max(1, len(d))
        res["valu"] = v
        # active lanes per issued VALU instruction (1.0 = no divergence)
        res["valu_lane_utilisation"] = v["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64.0 * v["SQ_ACTIVE_INST_VALU"])
        # (bench.py turns these into the VALU issue utilisation with its own live
        # kernel time: counter collection itself slows the dispatches ~3x)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
