#!/bin/bash
# One GPU-box session: parity tests, bench, other-config timings, rocprof kernel trace.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_fail() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "GPU step failed rc=$rc: stopping"; exit "$rc"; fi; }
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -30 gpurun_out/pytest_gpu.log; ok_or_fail $rc
fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --secondary > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; ok_or_fail $rc
if [ "${CONFIGS:-1}" = "1" ]; then
  timeout -k 10 300 python -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
  rc=$?; cat gpurun_out/configs.jsonl; tail -5 gpurun_out/configs.err; ok_or_fail $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?; tail -3 gpurun_out/prof.err; ok_or_fail $rc
  find gpurun_out/prof -name "*stats*"
fi
