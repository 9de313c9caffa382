set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
rc=$?; cat $O/bench_c4.json; exit $rc
