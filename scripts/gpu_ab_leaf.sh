#!/bin/bash
# Binary LBVH with leaf runs (RT0_BVH_LEAF=k: subtrees of <= k triangles become
# leaves): model parity tests (default and k=4, JIT and ahead-of-time kernels),
# then the C5 A/B of k.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/leaf
export TMPDIR=/tmp
for k in 1 4; do
  RT0_BVH_LEAF=$k timeout -k 10 600 python -u -m pytest tests/test_models.py -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/leaf/pytest_models_leaf$k.log 2>&1
  rc=$?; echo "leaf $k:"; tail -2 gpurun_out/leaf/pytest_models_leaf$k.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
CFG=c5 STEPS=2 AB="X=0
RT0_BVH_LEAF=2
RT0_BVH_LEAF=3
RT0_BVH_LEAF=4
RT0_BVH_LEAF=8
X=1" bash scripts/gpu_ab_env.sh
