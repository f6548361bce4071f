#!/bin/bash
# GPU call (round 5, batch 2): parity of the variant builds, C2 A/Bs of the tile variants,
# a C3 A/B of the 7-wave dense kernel, and the N = 8 shard rehearsal with the tick event.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CHECK="tglds s16 s32 d7 tickev" PAIRS="base3:tglds base3:s16 base3:s32" TAG=r5b2 bash tools/gpu_r5_variants.sh || exit 1
WL=c3 STEPS=20 ROUNDS=4 PAIRS="base3:d7" TAG=r5b2c3 bash tools/gpu_r5_ab.sh || exit 1
LIBS="base3 tickev" REPS=3 N=8 TAG=r5b2shard bash tools/gpu_r5_shard.sh || exit 1
