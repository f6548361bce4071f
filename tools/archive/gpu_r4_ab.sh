#!/bin/bash
# GPU call: interleaved A/B of library builds on C2 (tools/ab.py), per-kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4ab
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab.py --workload ${WL:-c2} --rounds ${ROUNDS:-6} --steps ${STEPS:-50} --per-kernel ${LIBS:-tools/ab_libs/base.so tools/ab_libs/passa_v2.so} > $OUT/ab_${TAG:-x}.txt 2>&1 || { tail -20 $OUT/ab_${TAG:-x}.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_${TAG:-x}.txt | tail -40
