#!/bin/bash
# A/B bench of the kernel variants (+ tests first). Stops at the first GPU fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_fail() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "GPU step failed rc=$rc: stopping"; exit "$rc"; fi; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_gpu.log; ok_or_fail $rc
fi
for v in ${VARIANTS:-"--jit 1" "--jit 0"}; do :; done
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $args > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  rc=$?; echo "== $args"; cat gpurun_out/ab_$i.json; tail -3 gpurun_out/ab_$i.err; ok_or_fail $rc
done <<< "${AB:-$'--jit 1\n--jit 0'}"
