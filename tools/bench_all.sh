#!/bin/bash
# Every bench workload once (one GPU), JSON lines into gpurun_out/bench_all/
# (c3 runs the hierarchy exchange by default; hier.json is c3 without it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench_all
for w in ${WORKLOADS:-c1 c1ps c2 c3 c4}; do
  timeout -k 10 600 python bench.py --workload $w --steps ${STEPS:-20} --warmup 3 $( [ "$w" = c1 ] || echo --no-cpu-baseline ) \
    > gpurun_out/bench_all/$w.json 2> gpurun_out/bench_all/$w.err
  s=$?; echo "$w status $s"; [ $s -ne 0 ] && { tail -3 gpurun_out/bench_all/$w.err; exit $s; }
done
timeout -k 10 600 python bench.py --workload c3 --hier off --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
  > gpurun_out/bench_all/hier.json 2> gpurun_out/bench_all/hier.err
s=$?; echo "c3 without hierarchy: status $s"; exit $s
