#!/bin/bash
# Where a pass kernel's wave cycles go: one rocprofv3 --pmc pass (8 SQ
# counters, kernel trace only) over a short bench run of workload $CFG.
# SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFG=${CFG:-c2}
O=gpurun_out/stall_$CFG${TAG:+_$TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/raw -o run -- \
  python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $O/run.log 2>&1
rc=$?; echo "stall pmc $CFG rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/run.log; exit $rc; }
python3 scripts/stall_summary.py $O/raw > $O/summary.txt; cat $O/summary.txt
