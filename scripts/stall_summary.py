#!/usr/bin/env python3
"""Sum the SQ stall counters of scripts/gpu_stall_pmc.sh per kernel (the pass
kernel's launches) and print the split of wave cycles."""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        k = row.get("Kernel_Name", "?")
        tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in tot.items():
    if "pass" not in k:
        continue
    w = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    print(k[:60])
    for n in sorted(c):
        print("  %-22s %16.4g  %6.3f of wave cycles" % (n, c[n], c[n] / w))
