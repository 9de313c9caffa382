set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -3 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
rc=$?; cat $O/bench_default.json; exit $rc
