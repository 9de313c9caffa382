set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  for cfg in c2 c3 c5 c4; do
    for v in base prev; do
      if [ $v = base ]; then
        timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/${cfg}_${v}_$round.json 2> $O/${cfg}_${v}_$round.err
      else
        timeout -k 10 300 env PROBES_PATCH=scripts/ab_r4_geomprev.patch bash scripts/probes.sh python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/${cfg}_${v}_$round.json 2> $O/${cfg}_${v}_$round.err
      fi
      rc=$?; echo "$cfg $v $round rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms_per_launch'], d.get('gpu_clock', {}).get('median_mhz'))" $O/${cfg}_${v}_$round.json 2>/dev/null)"
      if [ $rc -ne 0 ]; then tail -5 $O/${cfg}_${v}_$round.err; exit $rc; fi
    done
  done
done
exit 0
