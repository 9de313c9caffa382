#!/bin/bash
# The halo check compiled out of unsharded scene-specialised kernels: the GPU
# suite (sharded ReSTIR tests compile it in), then C3 / C5 against the round-2
# defaults before batching.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/halo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/halo/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/halo/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=c3 STEPS=5 AB="X=0
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1 RT0_JIT_WAVES_PER_EU=5
X=1
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1 RT0_JIT_WAVES_PER_EU=5" bash scripts/gpu_ab_env.sh || exit $?
CFG=c5 STEPS=2 AB="X=0" bash scripts/gpu_ab_env.sh
