#!/bin/bash
# Batched ReSTIR taps, second A/B: batch size at the ReSTIR occupancy target
# of 4 waves/SIMD, against the round-2 default (batch 1, 5 waves), on C3; C5
# (models: batch 1, 6 waves) must be unchanged.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=c3 STEPS=3 AB="X=0
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=1 RT0_JIT_WAVES_PER_EU=5
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=3
RT0_JIT_EXTRA=-DRT0_TAP_BATCH=4
X=1" bash scripts/gpu_ab_env.sh || exit $?
CFG=c5 STEPS=2 AB="X=0" bash scripts/gpu_ab_env.sh
