#!/bin/bash
# Round profile set for the bench workload: rocprofv3 kernel stats, then PMC
# passes (one rocprofv3 run each, --pmc with kernel trace only) summarised by
# scripts/pmc_traffic.py into gpurun_out/prof/pmc_summary.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
CMD="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats -o run --output-format csv -- $CMD > gpurun_out/prof/stats_bench.json 2> gpurun_out/prof/stats.err
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof/stats.err; exit $rc; }
i=0
for pass in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/prof/pmc$i -o run -- $CMD > gpurun_out/prof/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i ($pass): rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/prof/pmc$i.log; exit $rc; }
done
python3 scripts/pmc_traffic.py gpurun_out/prof/pmc1 gpurun_out/prof/pmc2 gpurun_out/prof/pmc_summary.json 1024 1024 gpurun_out/prof/pmc3
