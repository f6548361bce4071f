#!/bin/bash
# GPU call: configs[3]'s per-rank step at N = 2 / 4 / 8 shard sizes on one GPU
# (bench.py --rehearse-shard), with a kernel trace of the N = 8 step (tools/step_trace.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4shard
rm -rf $OUT; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py tests/test_large_gpu.py tests/test_c3_full_gpu.py tests/test_parity_gpu.py::test_arrivals_without_expiry_need_a_clock > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
fi
for n in ${SHARDS:-8 4 2}; do
  timeout -k 10 300 python -u bench.py --rehearse-shard $n --steps ${STEPS:-200} --warmup 5 > $OUT/shard$n.json 2> $OUT/shard$n.err || { tail -5 $OUT/shard$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/shard$n.json')); print($n, d['rehearsal']['step_us'], d['kernels'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --rehearse-shard 8 --steps 200 --warmup 5 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 tools/step_trace.py $OUT/trace --skip 60 --show 3 | tee $OUT/step_trace.txt
