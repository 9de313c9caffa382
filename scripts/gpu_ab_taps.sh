#!/bin/bash
# Batched ReSTIR tap loads (RT0_TAP_BATCH): the ReSTIR parity tests on the
# default, then the C3 / C5 A/B of batch size x occupancy target.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/taps
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_models.py tests/test_animated.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "restir or c5 or anim" > gpurun_out/taps/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/taps/pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for c in ${CFGS:-c3 c5}; do
  echo "=== $c"
  CFG=$c STEPS=2 AB="RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1
X=0
RT0_JIT_WAVES_PER_EU=4
RT0_JIT_WAVES_PER_EU=3
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=4 RT0_JIT_WAVES_PER_EU=3
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1" bash scripts/gpu_ab_env.sh || exit $?
done
