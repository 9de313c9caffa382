#!/bin/bash
# A/B of the XCD-aware tile order (RT0_XCD_REMAP, scene-specialised kernels)
# on every bench workload; prints Msamples/s and kernel ms per launch.
mkdir -p gpurun_out/ab_xcd
for cfg in ${CONFIGS:-c3 c5 c2 c4}; do for X in ${MODES:-0 1 4 16}; do
  st=5; [ $cfg = c5 ] && st=3
  RT0_JIT_EXTRA="-DRT0_XCD_REMAP=$X" timeout -k 10 200 python bench.py --config $cfg --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/ab_xcd/bench_${cfg}_X$X.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_xcd/bench_${cfg}_X$X.json'));print('$cfg remap=$X',d['value'],d['roofline']['kernel_ms_per_launch'])"
done; done
