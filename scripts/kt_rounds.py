"""Per-dispatch durations of the last wavefront launch in a kernel trace:
    kt_rounds.py TRACE_DIR [LAUNCHES]   (S = shade, P = plan, M = march, us)"""
import csv
import glob
import sys

rows = []
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(fn)))
rows.sort(key=lambda r: float(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].strip(), float(r["Start_Timestamp"]), float(r["End_Timestamp"])) for r in rows
       if r["Kernel_Name"].strip().startswith("rt0_jit_wf")]
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 3
last = seq[-len(seq) // nl:]
print(" ".join("%s%.0f" % (k[11].upper(), (e - s) / 1e3) for k, s, e in last))
print("span of the launch: %.3f ms, kernels %.3f ms" % ((last[-1][2] - last[0][1]) / 1e6,
                                                       sum(e - s for _, s, e in last) / 1e6))
