#!/bin/bash
# 4-wide vs binary BVH walk on C5: kernel resources (rocprofv3 kernel trace:
# VGPRs, LDS, scratch) of both, then the occupancy-target A/B of the 4-wide walk.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bvh4b
export TMPDIR=/tmp
for w in 1 0; do
  RT0_BVH_DEBUG=1 RT0_BVH_WIDE=$w timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bvh4b/kt_w$w -o run -- \
    python bench.py --config ${CFG:-c5} --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bvh4b/kt_w$w.json 2> gpurun_out/bvh4b/kt_w$w.err
  rc=$?; echo "kernel trace wide=$w rc=$rc"; grep "rt0 bvh" gpurun_out/bvh4b/kt_w$w.err | head -2
  [ $rc -ne 0 ] && { tail -5 gpurun_out/bvh4b/kt_w$w.err; exit $rc; }
  python3 - gpurun_out/bvh4b/kt_w$w <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rt0_jit_pass" in r.get("Kernel_Name", "")]
r = rows[-1]
print({k: r[k] for k in r if any(s in k for s in ("VGPR", "SGPR", "LDS", "Scratch", "Workgroup_Size"))})
EOF
done
STEPS=2 CFG=${CFG:-c5} AB="RT0_JIT_WAVES_PER_EU=5
RT0_JIT_WAVES_PER_EU=4
RT0_JIT_WAVES_PER_EU=3
RT0_BVH_LEAF=2 RT0_JIT_WAVES_PER_EU=4" bash scripts/gpu_ab_env.sh
