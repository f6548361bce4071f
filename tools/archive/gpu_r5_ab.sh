#!/bin/bash
# GPU call (round 5): interleaved A/B runs of library builds (tools/ab.py), two builds
# per process, each pair in both orders.  PAIRS="a:b c:d" names builds in tools/ab_libs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p $OUT
for pr in ${PAIRS:-base:exp1}; do
  a=${pr%%:*}; b=${pr##*:}
  for order in "$a $b" "$b $a"; do
    set -- $order
    f=$OUT/ab_${1}_${2}.txt
    timeout -k 10 300 python -u tools/ab.py --workload ${WL:-c2} --rounds ${ROUNDS:-6} --steps ${STEPS:-50} --per-kernel \
      tools/ab_libs/$1.so tools/ab_libs/$2.so > $f 2>&1 || { tail -20 $f; exit 1; }
    grep -v amdgpu.ids $f | tail -4
  done
done
