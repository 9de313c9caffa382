#!/bin/bash
# Round-2 session-3 GPU pass: the full GPU suite on the defaults, then A/B of
# the shadow-ray light test on C2 and the ReSTIR spatial-tap locality bound on C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2s3
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r2s3/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r2s3/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c2 AB="X=0
RT0_JIT_EXTRA=-DRT0_FAST_SHADOW=0
X=0
RT0_JIT_EXTRA=-DRT0_FAST_SHADOW=0" bash scripts/gpu_ab_env.sh || exit $?
CFG=c3 AB="X=0
RT0_JIT_EXTRA=-DRT0_EXP_SPATIAL_SELF
X=0
RT0_JIT_EXTRA=-DRT0_EXP_SPATIAL_SELF" bash scripts/gpu_ab_env.sh
