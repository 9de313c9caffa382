#!/bin/bash
# One GPU-box session: parity tests, the bench line of each BASELINE workload,
# steady-state kernel times (rocprofv3 --kernel-trace), PMC passes, A/B
# variants and the FETCH_SIZE calibration.  Replaces round 2's gpu_round2.sh,
# gpu_pmc.sh, gpu_stall_pmc.sh and the 25 one-off gpu_ab_*.sh scripts.
# Every GPU step runs under its own time limit; the script stops at the first
# step that faults, aborts or times out (exit codes other than 0/1).
#
# Env (all optional):
#   OUT=name          results under gpurun_out/<name>/
#   TESTS=1|0         python -m pytest tests -m gpu (PYTEST_K = a -k expression)
#   CONFIGS="c2 c1 c3 c4 c5"   STEPS=5 WARMUP=2
#   BENCH=1|0         plain bench line per config
#   PROFILE=1|0       rocprofv3 --kernel-trace of a bench run -> steady-state kernel time
#   PMC=1|0           counter passes: FETCH_SIZE | WRITE_SIZE | VALU + GRBM clock | SQ stall split
#                     (MIX=1 adds the VALU instruction-mix pass: ADD/MUL/FMA/TRANS/INT32/CVT)
#   AB="name:VAR=val VAR2=val;name2:VAR=val"  bench every config under each
#                     variant (env assignments), ROUNDS interleaved rounds, plus
#                     the default ("base") in every round; AB_CONFIGS overrides CONFIGS
#   CALIB=1           scripts/fetch_calib under rocprofv3 --pmc FETCH_SIZE, and
#                     scripts/valu_peak (measured scalar / packed FP32 FMA peaks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-measure}
mkdir -p "$O"
export TMPDIR=/tmp
export RT0_SEGV_TRACE=1  # librt0 prints the native stack of a segmentation fault (rt0_host.cpp)
STEPS=${STEPS:-5}
WARMUP=${WARMUP:-2}

stop_if_bad() {  # $1 = rc of a GPU step; 0 ok, 1 = test failures (keep going)
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step failed rc=$1: stopping"; exit "$1"; fi
}
declare -A BPP=([c1]=32 [c2]=32 [c2_refcaps]=32 [c3]=160 [c4]=32 [c5]=160)
declare -A WH=([c1]="256 256" [c2]="1024 1024" [c2_refcaps]="1024 1024" [c3]="1920 1080" [c4]="2048 2048" [c5]="4096 4096")
declare -A LPS=([c1]=1 [c2]=1 [c2_refcaps]=1 [c3]=16 [c4]=1 [c5]=4)  # pass launches per bench step

if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -25 "$O/pytest_gpu.log"; stop_if_bad $rc
fi

if [ "${CALIB:-0}" = "1" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/calib" -o run -- \
    ./scripts/fetch_calib > "$O/calib.log" 2>&1
  rc=$?; echo "calib rc=$rc"; tail -2 "$O/calib.log"; stop_if_bad $rc
  python3 scripts/fetch_calib.py "$O/calib" "$O/calib.log" > "$O/calib.json"; cat "$O/calib.json"
  # measured FP32 VALU peaks: scalar v_fma_f32 vs packed v_pk_fma_f32
  timeout -k 10 60 ./scripts/valu_peak > "$O/valu_peak.json" 2>&1
  rc=$?; echo "valu peak rc=$rc"; cat "$O/valu_peak.json"; stop_if_bad $rc
fi

# dispatches per kernel per ReSTIR pass: K where librt0 splits the pass into
# K row parts (rt0_host.cpp restir_split_parts: 3 for scenes with models, i.e.
# c5, unless RT0_RESTIR_SPLIT says otherwise)
halves() {
  if [ -n "${RT0_RESTIR_SPLIT:-}" ]; then
    k=$RT0_RESTIR_SPLIT; [ "$k" = "1" ] && k=2; [ "$k" -gt 4 ] && k=4
    { [ "$k" != "0" ] && [ "$1" = "c3" -o "$1" = "c5" ]; } && echo $k || echo 1
  else
    [ "$1" = "c5" ] && echo 3 || echo 1
  fi
}
for cfg in ${CONFIGS:-c2 c1 c3 c4 c5}; do
  if [ "${BENCH:-1}" = "1" ]; then
    extra=""; [ "$cfg" = "c2" ] && extra="--secondary"
    timeout -k 10 300 python bench.py --config $cfg --steps $STEPS --warmup $WARMUP $extra > "$O/bench_$cfg.json" 2> "$O/bench_$cfg.err"
    rc=$?; cat "$O/bench_$cfg.json"; tail -3 "$O/bench_$cfg.err"; stop_if_bad $rc
  fi
  skip=$((WARMUP * ${LPS[$cfg]}))
  if [ "${PROFILE:-1}" = "1" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$cfg" -o run -- \
      python bench.py --config $cfg --steps $STEPS --warmup $WARMUP --no-cpu-baseline --no-secondary > "$O/prof_$cfg.json" 2> "$O/prof_$cfg.err"
    rc=$?; echo "kernel trace $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/prof_$cfg.err"; exit $rc; }
    HALVES=$(halves $cfg) python3 scripts/kt_summary.py "$O/kt_$cfg.json" "$O/kt_$cfg" $skip
    find "$O/kt_$cfg" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_$cfg.csv" \;
    rm -rf "$O/kt_$cfg"
  fi
  if [ "${PMC:-1}" = "1" ]; then
    # one warm-up step + one counted step; the warm-up's dispatches are skipped
    CMD="python bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-secondary"
    i=0; dirs=""
    for pass in "FETCH_SIZE" "WRITE_SIZE" \
        "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" \
        ${MIX:+"SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SMEM"}; do
      i=$((i+1))
      timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$O/pmc_${cfg}_$i" -o run -- $CMD > "$O/pmc_${cfg}_$i.log" 2>&1
      rc=$?; echo "pmc $cfg pass $i: rc=$rc"
      [ $rc -ne 0 ] && { tail -5 "$O/pmc_${cfg}_$i.log"; exit $rc; }
      dirs="$dirs $O/pmc_${cfg}_$i"
    done
    HALVES=$(halves $cfg) python3 scripts/pmc_summary.py "$O/pmc_$cfg.json" ${WH[$cfg]} ${BPP[$cfg]} ${LPS[$cfg]} $dirs
    rm -rf $dirs
  fi
done

if [ -n "${AB:-}" ]; then
  IFS=';' read -ra VARS <<< "base:;$AB"
  for round in $(seq 1 ${ROUNDS:-2}); do
    for cfg in ${AB_CONFIGS:-${CONFIGS:-c2 c1 c3 c4 c5}}; do
      for v in "${VARS[@]}"; do
        name=${v%%:*}; envs=${v#*:}
        timeout -k 10 300 env $envs python bench.py --config $cfg --steps $STEPS --warmup $WARMUP --no-cpu-baseline --no-secondary \
          > "$O/ab_${cfg}_${name}_r$round.json" 2> "$O/ab_${cfg}_${name}_r$round.err"
        rc=$?; echo "ab $cfg $name round $round rc=$rc: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['events_per_sample'].get('bvh_node'), d.get('gpu_clock', {}).get('median_mhz'))" "$O/ab_${cfg}_${name}_r$round.json" 2>/dev/null)"
        stop_if_bad $rc
      done
    done
  done
fi
echo "gpu_measure done"
