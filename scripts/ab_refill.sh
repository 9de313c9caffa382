mkdir -p gpurun_out/r2f
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2f/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r2f/pytest_gpu.log
grep -E "FAILED|ERROR" gpurun_out/r2f/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
for cfg in c3 c5; do for R in 1 2 4; do
  st=5; [ $cfg = c5 ] && st=3
  RT0_REFILL=$R timeout -k 10 200 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/r2f/bench_${cfg}_R$R.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r2f/bench_${cfg}_R$R.json'));print('$cfg R=$R',d['value'],d['roofline']['kernel_ms_per_launch'])"
done; done
