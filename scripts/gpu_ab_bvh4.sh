#!/bin/bash
# 4-wide BVH: the model parity tests on the default (4-wide) walk, then the
# C5 A/B of the walk (binary vs 4-wide) and of the collapse's leaf size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bvh4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_models.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/bvh4/pytest_models.log 2>&1
rc=$?; tail -15 gpurun_out/bvh4/pytest_models.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
CFG=${CFG:-c5} STEPS=${STEPS:-2} AB="${AB:-X=0
RT0_BVH_WIDE=0
RT0_BVH_LEAF=2
RT0_BVH_LEAF=4
X=1}" bash scripts/gpu_ab_env.sh
