#!/bin/bash
# Wave-uniform material lookups (RT0_JIT_UMAT): parity tests with the knob,
# then C2 / C4 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/umat
export TMPDIR=/tmp
RT0_JIT_UMAT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/umat/pytest_parity.log 2>&1
rc=$?; tail -2 gpurun_out/umat/pytest_parity.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c2 STEPS=10 AB="X=0
RT0_JIT_UMAT=1
X=1
RT0_JIT_UMAT=1" bash scripts/gpu_ab_env.sh || exit $?
CFG=c4 STEPS=2 AB="X=0
RT0_JIT_UMAT=1" bash scripts/gpu_ab_env.sh
