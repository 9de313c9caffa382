set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
export TMPDIR=/tmp RT0_SEGV_TRACE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
# the pooled closest-hit walks (RT0_WALK_POOL) against the model tests
RT0_JIT_EXTRA=-DRT0_WALK_POOL=1 timeout -k 10 400 python -u -m pytest tests/test_models.py tests/test_gpu_defer.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_walkpool.log 2>&1
rc=$?; tail -3 $O/pytest_walkpool.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
ab() {  # config name env...
  cfg=$1; name=$2; shift 2
  timeout -k 10 300 env "$@" python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/ab_${cfg}_$name.json 2> $O/ab_${cfg}_$name.err
  rc=$?; echo "ab $cfg $name rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], d['gpu_clock'].get('median_mhz'))" $O/ab_${cfg}_$name.json 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -5 $O/ab_${cfg}_$name.err; exit $rc; }
  return 0
}
ab c4 base X=1 && ab c4 nopool RT0_JIT_EXTRA=-DRT0_MARCH_POOL=0 && ab c4 b4 RT0_JIT_EXTRA=-DRT0_MARCH_BUDGET=4 && ab c4 b16 RT0_JIT_EXTRA=-DRT0_MARCH_BUDGET=16 && ab c4 base2 X=1 || exit $?
ab c5 base X=1 && ab c5 wpool RT0_JIT_EXTRA=-DRT0_WALK_POOL=1 && ab c5 wpool6 RT0_JIT_EXTRA=-DRT0_WALK_POOL=1 RT0_JIT_WAVES_PER_EU=6 && ab c5 wpool_b16 "RT0_JIT_EXTRA=-DRT0_WALK_POOL=1 -DRT0_WALK_BUDGET=16" && ab c5 tap2 RT0_JIT_EXTRA=-DRT0_TAP_BATCH=2 && ab c5 base2 X=1 || exit $?
ab c2 base X=1 && ab c2 pk RT0_JIT_EXTRA=-DRT0_PK_GEOM=1 && ab c2 base2 X=1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err; echo "c2 rc=$?"; head -c 400 $O/bench_c2.json
