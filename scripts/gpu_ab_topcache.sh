#!/bin/bash
# Stack-top node cache of the BVH walk (RT0_BVH_TOPCACHE, binary16 nodes):
# model parity tests with the knob on, then the C5 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/topcache
export TMPDIR=/tmp
RT0_JIT_EXTRA=-DRT0_BVH_TOPCACHE=1 timeout -k 10 600 python -u -m pytest tests/test_models.py -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/topcache/pytest_models.log 2>&1
rc=$?; tail -3 gpurun_out/topcache/pytest_models.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c5 STEPS=2 AB="X=0
RT0_JIT_EXTRA=-DRT0_BVH_TOPCACHE=1
RT0_JIT_EXTRA=-DRT0_BVH_TOPCACHE=1 RT0_JIT_WAVES_PER_EU=5
X=1
RT0_JIT_EXTRA=-DRT0_BVH_TOPCACHE=1" bash scripts/gpu_ab_env.sh
