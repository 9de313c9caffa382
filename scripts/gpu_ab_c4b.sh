#!/bin/bash
# Full GPU suite on the current build, then the C4 march-slice length A/B
# (RT0_MARCH_BUDGET steps per slice of the wave's one sphere-tracing loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c4b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c4b/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/c4b/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c4 STEPS=3 AB="X=0
RT0_JIT_EXTRA=-DRT0_MARCH_BUDGET=4
RT0_JIT_EXTRA=-DRT0_MARCH_BUDGET=16
RT0_JIT_EXTRA=-DRT0_MARCH_BUDGET=32
X=1" bash scripts/gpu_ab_env.sh
