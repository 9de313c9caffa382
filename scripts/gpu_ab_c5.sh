#!/bin/bash
# C5 occlusion-query A/B (and the GPU model tests on the defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_models.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/ab5/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ab5/pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c5 STEPS=2 AB="X=0
RT0_JIT_EXTRA=-DRT0_FAST_SHADOW=0
X=0
RT0_JIT_EXTRA=-DRT0_EXP_NO_SHADOW" bash scripts/gpu_ab_env.sh
