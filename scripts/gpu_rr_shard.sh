#!/bin/bash
# Round-robin ReSTIR bands: the whole GPU suite (incl. the round-robin shard
# test), then the load-balance simulation of contiguous vs round-robin splits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rr
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/rr/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/rr/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python scripts/restir_shard_sim.py c3 c5 > gpurun_out/rr/shard_sim.log 2>&1
rc=$?; cat gpurun_out/rr/shard_sim.log | grep -v "^{"; exit $rc
