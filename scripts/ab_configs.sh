#!/bin/bash
# A/B of JIT knobs on the other BASELINE configs (scripts/bench_configs.py):
# each line of $AB is a set of env assignments; $RUNS selects the configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
while read -r line; do
  [ -z "$line" ] && continue
  env $line timeout -k 10 200 python scripts/bench_configs.py --runs "${RUNS:-c3,c4,c5}" --steps 2 > gpurun_out/abc.jsonl 2>&1
  echo "== [$line] rc=$? $(python3 -c "
import json
for l in open('gpurun_out/abc.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['config'], d['kernel_ms_per_step'], end='  ')
")"
done <<< "$AB"
