#!/bin/bash
# GPU call (round 5): parity of A/B builds against the oracle (tools/variant_check.py),
# then interleaved A/B timings (tools/gpu_r5_ab.sh).  CHECK="a b" and PAIRS="base:a ..."
# name builds in tools/ab_libs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5var}
mkdir -p $OUT
libs=""; for v in ${CHECK:-}; do libs="$libs tools/ab_libs/$v.so"; done
if [ -n "$libs" ]; then
  timeout -k 10 600 python -u tools/variant_check.py $libs > $OUT/check.txt 2>&1 || { tail -30 $OUT/check.txt; exit 1; }
  grep -v amdgpu.ids $OUT/check.txt
fi
TAG=${TAG:-r5var} bash tools/gpu_r5_ab.sh
