#!/bin/bash
# GPU call: default bench (C3 + hierarchy + C1 extra + CPU baseline) and the
# spawned 2-rank rehearsal on one GPU.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  s=$?; tail -3 gpurun_out/pytest_gpu.log; [ $s -ne 0 ] && exit $s
fi
timeout -k 10 400 python -u bench.py --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
s=$?; cat gpurun_out/bench_default.json; tail -3 gpurun_out/bench_default.err; [ $s -ne 0 ] && exit $s
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 --warmup 3 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
s=$?; cat gpurun_out/bench_g2.json; tail -3 gpurun_out/bench_g2.err; exit $s
