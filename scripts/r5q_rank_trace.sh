cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r5q
for cfg in "1 1" "0 8"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5q/kt_$1_$2 -o run -- python3 scripts/shard_trace.py c5 $1 $2 64 > gpurun_out/r5q/log_$1_$2.txt 2>&1 || exit 3
  python3 - gpurun_out/r5q/kt_$1_$2 <<'PY'
import csv, glob, sys, collections
rows=[]
for fn in glob.glob(sys.argv[1]+"/**/*kernel_trace.csv", recursive=True): rows+=list(csv.DictReader(open(fn)))
rows.sort(key=lambda r: float(r["Start_Timestamp"]))
ks=[r for r in rows if r["Kernel_Name"].startswith("rt0_jit")]
last=ks[-4:]
t0=float(last[0]["Start_Timestamp"])
for r in last:
    print(r["Kernel_Name"][:16], "start %.3f dur %.3f" % ((float(r["Start_Timestamp"])-t0)/1e6, (float(r["End_Timestamp"])-float(r["Start_Timestamp"]))/1e6))
PY
done
