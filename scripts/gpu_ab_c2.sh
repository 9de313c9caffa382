#!/bin/bash
# Round-2 session 3 A/B on the headline kernel: parity of every knob at once,
# then the bench per knob, then the stall counters of the default kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab2
export TMPDIR=/tmp
ALL="RT0_JIT_EXTRA=-DRT0_OPQ=0,-DRT0_TYPE_BITS=1,-DRT0_CAM_RCP=1"
env $ALL timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_props.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab2/pytest_knobs.log 2>&1
rc=$?; tail -4 gpurun_out/ab2/pytest_knobs.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
AB="X=0
RT0_JIT_EXTRA=-DRT0_OPQ=0
RT0_JIT_EXTRA=-DRT0_TYPE_BITS=1
RT0_JIT_EXTRA=-DRT0_CAM_RCP=1
RT0_PERSIST=2048
RT0_PERSIST=1024
$ALL RT0_PERSIST=2048
X=0" bash scripts/gpu_ab_env.sh || exit $?
bash scripts/gpu_stall_pmc.sh
