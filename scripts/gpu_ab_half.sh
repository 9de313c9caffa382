#!/bin/bash
# binary16 BVH nodes (RT0_BVH_HALF): model parity tests with the knob on in
# the scene-specialised kernels, then the C5 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/half
export TMPDIR=/tmp
RT0_JIT_EXTRA=-DRT0_BVH_HALF=1 timeout -k 10 600 python -u -m pytest tests/test_models.py -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/half/pytest_models_half.log 2>&1
rc=$?; tail -3 gpurun_out/half/pytest_models_half.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c5 STEPS=2 AB="X=0
RT0_JIT_EXTRA=-DRT0_BVH_HALF=1
X=1
RT0_JIT_EXTRA=-DRT0_BVH_HALF=1 RT0_JIT_WAVES_PER_EU=5" bash scripts/gpu_ab_env.sh
# the model's share of C5 at 1024^2: the icosphere through the BVH vs an analytic sphere
timeout -k 10 300 python scripts/probe_c5.py
