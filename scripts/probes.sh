#!/bin/bash
# Profiling probes (parity-breaking, never in the product source): applies
# scripts/probes.patch to a scratch copy of the integrator, writes the JIT
# device source (rt0_device.h + patched rt0_integrator.h, as tools_embed.py
# concatenates them) and runs the given command with RT0_JIT_SOURCE pointing
# at it.  Choose the probe with RT0_JIT_EXTRA, e.g.
#   scripts/probes.sh env RT0_JIT_EXTRA=-DRT0_EXP_NO_NEE python scripts/exp_c4.py 1024 8 causes
# Probes: RT0_EXP_NO_BVH_OCC, RT0_EXP_NO_SHADOW, RT0_EXP_SPATIAL_SELF,
# RT0_EXP_NO_NEE, RT0_EXP_NO_VOL_NEE, RT0_NO_MIS_REUSE, RT0_FAST_SHADOW=0.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$(mktemp -d)
cp raytracer-0_amd/csrc/rt0_device.h raytracer-0_amd/csrc/rt0_integrator.h "$T/"
patch -s -d "$T" -p3 < "${PROBES_PATCH:-scripts/probes.patch}"
cat "$T/rt0_device.h" "$T/rt0_integrator.h" > "$T/rt0_jit_probe.src"
export RT0_JIT_SOURCE="$T/rt0_jit_probe.src"
"$@"
