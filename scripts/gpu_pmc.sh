#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --pmc only with kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
CMD="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for pass in "${@:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i ($pass): rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
