#!/bin/bash
# Kernel traces of one workload under several environment variants (A/B of
# per-kernel times): scripts/kt_compare.sh OUT CONFIG "name:VAR=val VAR2=val" ...
# -> gpurun_out/OUT/kt_<name>.json (scripts/kt_summary.py, warm-up launch skipped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1; cfg=$2; shift 2
mkdir -p "$O"
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$name" -o run -- \
    python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > "$O/kt_$name.log" 2>&1
  rc=$?; echo "kt $name rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/kt_$name.log"; exit $rc; }
  python3 scripts/kt_summary.py "$O/kt_$name.json" "$O/kt_$name" 1
  python3 - "$O/kt_$name" <<'PY'
import csv, glob, sys, collections
rows = []
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(fn)))
rows.sort(key=lambda r: float(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].strip()[:24], (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3) for r in rows
       if r["Kernel_Name"].strip().startswith("rt0_jit_wf")]
n = len(seq) // 3  # three launches (warm-up + 2): the last one's rounds
print(" ".join("%s%.0f" % ("S" if k.endswith("shade") else "M", us) for k, us in seq[-n:]))
PY
  rm -rf "$O/kt_$name"
done
