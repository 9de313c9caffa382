set -o pipefail
export TMPDIR=/tmp RT0_SEGV_TRACE=1
OUT=r04i TESTS=1 CONFIGS="c2 c1 c3 c4 c5" MIX=1 bash scripts/gpu_measure.sh
