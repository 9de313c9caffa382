set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp RT0_SEGV_TRACE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -6 $O/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
OUT=r04 TESTS=0 CONFIGS="${CONFIGS:-c2 c1 c3}" MIX=1 bash scripts/gpu_measure.sh
