set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
RT0_JIT_EXTRA=-DRT0_MARCH_FLAT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_flat.log 2>&1
rc=$?; tail -4 $O/pytest_gpu_flat.log; [ $rc -gt 1 ] && exit $rc
OUT=r4j TESTS=0 BENCH=0 PROFILE=0 PMC=0 CONFIGS="c4" AB="flat:RT0_JIT_EXTRA=-DRT0_MARCH_FLAT=1" ROUNDS=3 bash scripts/gpu_measure.sh
