#!/bin/bash
# GPU suite on the defaults, then the occlusion-query A/B on C5 and C3 and the
# C2 default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2s4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r2s4/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r2s4/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c5 STEPS=2 AB="X=0
RT0_JIT_EXTRA=-DRT0_FAST_SHADOW=0
X=0" bash scripts/gpu_ab_env.sh || exit $?
CFG=c3 AB="X=0
RT0_JIT_EXTRA=-DRT0_FAST_SHADOW=0" bash scripts/gpu_ab_env.sh || exit $?
CFG=c2 AB="X=0" bash scripts/gpu_ab_env.sh
