#!/bin/bash
# C4 (Mandelbulb + volume) march-scheduling A/B: the full GPU suite on the
# defaults, the SDF/volumetric parity tests with the knobs on, then the C4
# bench per knob and the C2 bench on the defaults.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ab4/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/ab4/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
env RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=32,-DRT0_BULB_NOBREAK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -x -q -k "sdf or menger or mandel or vol or cone or prism or page" --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/ab4/pytest_knobs.log 2>&1
rc=$?; tail -4 gpurun_out/ab4/pytest_knobs.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c4 STEPS=3 AB="X=0
RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=32
RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=16
RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=48
RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=32,-DRT0_MARCH_BUDGET=2
RT0_JIT_EXTRA=-DRT0_MARCH_QUORUM=16,-DRT0_MARCH_BUDGET=4
RT0_JIT_EXTRA=-DRT0_BULB_NOBREAK=1
X=0" bash scripts/gpu_ab_env.sh || exit $?
CFG=c2 AB="X=0
X=1" bash scripts/gpu_ab_env.sh
