#!/bin/bash
# rocprofv3 evidence for one workload: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md §HBM / rocprofv3),
# plus the same counters on tools/ubench's flat8 kernel whose bytes are known
# (calibration for 8-byte-per-lane access).  Every step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-c1}
STEPS=${STEPS:-20}
OUT=gpurun_out/prof_$W
rm -rf $OUT; mkdir -p $OUT
run() {  # $1 = tag, rest = rocprofv3 args before --
  local tag=$1; shift
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d $OUT/$tag -o run -- \
    python3 bench.py --steps $STEPS --warmup 3 --workload $W --no-cpu-baseline --no-extra --no-busy-probe > $OUT/$tag.log 2>&1
  local s=$?
  if [ $s -ne 0 ]; then echo "STOP: $tag status $s"; tail -5 $OUT/$tag.log; exit $s; fi
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
if [ -x tools/ubench ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- ./tools/ubench 10000000 1000 > $OUT/cal_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- ./tools/ubench 10000000 1000 > $OUT/cal_write.log 2>&1 || exit $?
fi
python3 tools/pmc_summary.py $OUT $W
cp profiles/pmc_$W.json profiles/rocprof_$W.md $OUT/ && echo "summaries in $OUT"
