#!/bin/bash
# GPU call (round 6): rocprof kernel trace + PMC passes of the benched tree for the
# given workloads (tools/gpu_profile.sh each), then the default bench line.
# Every step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6prof}
mkdir -p $OUT
for w in ${WORKLOADS:-c3 c1}; do
  WORKLOAD=$w STEPS=${STEPS:-20} bash tools/gpu_profile.sh > $OUT/prof_$w.txt 2>&1 || { tail -20 $OUT/prof_$w.txt; exit 1; }
  cp -r gpurun_out/prof_$w $OUT/ 2>/dev/null
  echo "profiled $w"
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -8 $OUT/bench_default.err; exit 1; }
  tail -c 600 $OUT/bench_default.json
fi
