#!/bin/bash
# One GPU-box session of round 2: parity tests, the bench line of every
# BASELINE workload, rocprofv3 kernel stats and PMC passes per workload.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
# Env: TESTS=0 skips pytest; CONFIGS="c2 c1 c3 c4 c5" picks workloads;
#      PROFILE=0 skips rocprof; PMC=0 skips the counter passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r2}
mkdir -p $O
export TMPDIR=/tmp

ok_or_fail() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "GPU step failed rc=$rc: stopping"; exit "$rc"; fi; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
  rc=$?; tail -30 $O/pytest_gpu.log; ok_or_fail $rc
fi
declare -A BPP=([c1]=32 [c2]=32 [c2_refcaps]=32 [c3]=160 [c4]=32 [c5]=160)
declare -A WH=([c1]="256 256" [c2]="1024 1024" [c2_refcaps]="1024 1024" [c3]="1920 1080" [c4]="2048 2048" [c5]="4096 4096")
for cfg in ${CONFIGS:-c2 c1 c3 c4 c5}; do
  extra=""; [ "$cfg" = "c2" ] && extra="--secondary"
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-5} --warmup 1 $extra > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  rc=$?; cat $O/bench_$cfg.json; tail -3 $O/bench_$cfg.err; ok_or_fail $rc
  [ "${PROFILE:-1}" = "1" ] || continue
  CMD="python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- $CMD > $O/prof_$cfg.json 2> $O/prof_$cfg.err
  rc=$?; echo "stats $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/prof_$cfg.err; exit $rc; }
  [ "${PMC:-1}" = "1" ] || continue
  CMD="python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline"
  i=0
  for pass in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $O/pmc_${cfg}_$i -o run -- $CMD > $O/pmc_${cfg}_$i.log 2>&1
    rc=$?; echo "pmc $cfg pass $i ($pass): rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/pmc_${cfg}_$i.log; exit $rc; }
  done
  python3 scripts/pmc_traffic.py $O/pmc_${cfg}_1 $O/pmc_${cfg}_2 $O/pmc_$cfg.json ${WH[$cfg]} $O/pmc_${cfg}_3 ${BPP[$cfg]} > /dev/null
  # keep the merged-back output small: drop the raw counter CSVs once summarised
  rm -rf $O/pmc_${cfg}_1 $O/pmc_${cfg}_2 $O/pmc_${cfg}_3
done
find $O -name "*kernel_stats.csv" | sort
