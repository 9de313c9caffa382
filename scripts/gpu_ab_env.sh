#!/bin/bash
# A/B of JIT tuning knobs on the bench workload: each line of $AB is a set of
# env assignments (no spaces inside a value; RT0_JIT_EXTRA takes ',' lists).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  env $line timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/abenv_$i.json 2> gpurun_out/abenv_$i.err
  rc=$?
  echo "== [$line] rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/abenv_$i.json')); print(d['value'], d['roofline']['kernel_ms_per_launch'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/abenv_$i.err; exit $rc; fi
done <<< "${AB:-X=0}"
