#!/usr/bin/env python3
"""FETCH_SIZE calibration from scripts/fetch_calib (run under rocprofv3 --pmc
FETCH_SIZE by scripts/gpu_measure.sh CALIB=1): per access shape, the true HBM
bytes read (each kernel reads a 1 GiB table exactly once) over FETCH_SIZE x
1024 B = the factor that turns the counter into bytes for that shape.

    fetch_calib.py PMC_DIR CALIB_LOG
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, log = sys.argv[1], sys.argv[2]
    truth = json.loads([l for l in open(log) if l.startswith("{")][-1])
    per = defaultdict(list)
    for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        rows = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] == "FETCH_SIZE":
                rows[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        for i in sorted(rows):
            for k in truth:
                if k in names[i]:
                    per[k].append(rows[i] * 1024.0)
    out = {}
    for k, b in truth.items():
        f = per.get(k, [])
        out[k] = {"true_bytes": b, "fetch_size_bytes": f,
                  "factor": [round(b / x, 3) if x else None for x in f]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
