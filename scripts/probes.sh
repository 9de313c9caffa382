#!/bin/bash
# Profiling probes (parity-breaking, never in the product source or the
# product library): copies the repository to a scratch directory, applies
# scripts/probes.patch (or $PROBES_PATCH) to that copy's integrator, builds the
# copy's librt0.so there and runs the given command from inside the copy, so
# the command loads the probe library and the product tree stays untouched.
# Choose the probe with RT0_JIT_EXTRA, e.g.
#   scripts/probes.sh env RT0_JIT_EXTRA=-DRT0_EXP_NO_NEE python scripts/exp_c4.py 1024 8 causes
# Probes: RT0_EXP_NO_BVH_OCC, RT0_EXP_NO_SHADOW, RT0_EXP_SPATIAL_SELF,
# RT0_EXP_NO_NEE, RT0_EXP_NO_VOL_NEE, RT0_NO_MIS_REUSE, RT0_FAST_SHADOW=0.
# Output written under the copy's gpurun_out/ is copied back to this tree's.
set -e
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
T=$(mktemp -d)
tar -C "$ROOT" --exclude=./gpurun_out --exclude=./.git --exclude=./profiles --exclude='*.o' -cf - . | tar -C "$T" -xf -
patch -s -d "$T" -p1 < "${PROBES_PATCH:-scripts/probes.patch}"
( while sleep 30; do echo "probes.sh: building the probe library"; done ) & HB=$!
make -s -j16 -C "$T/raytracer-0_amd" rt0/librt0.so || { kill $HB; exit 1; }
kill $HB
mkdir -p "$T/gpurun_out"
rc=0
(cd "$T" && "$@") || rc=$?
mkdir -p "$ROOT/gpurun_out"
cp -r "$T/gpurun_out/." "$ROOT/gpurun_out/" 2>/dev/null || true
rm -rf "$T"
exit $rc
