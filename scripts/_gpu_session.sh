set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
O=gpurun_out/r4i; mkdir -p $O
RT0_PIX_QUEUE=4 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_q4.log 2>&1
rc=$?; tail -6 $O/pytest_gpu_q4.log; [ $rc -gt 1 ] && exit $rc
OUT=r4i TESTS=0 BENCH=0 PROFILE=0 PMC=0 CONFIGS="c4 c2 c1" AB="q2:RT0_PIX_QUEUE=2;q4:RT0_PIX_QUEUE=4" ROUNDS=2 bash scripts/gpu_measure.sh || exit $?
timeout -k 10 400 python -u scripts/restir_shard_sim.py c5 > $O/restir_shard_sim.txt 2>&1
rc=$?; tail -12 $O/restir_shard_sim.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/shard_sim.py > $O/shard_sim.txt 2>&1
rc=$?; cat $O/shard_sim.txt; exit $rc
