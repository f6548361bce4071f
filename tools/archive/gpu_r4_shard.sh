#!/bin/bash
# GPU call: configs[3]'s per-rank step at N = 8 / 4 / 2 shard sizes on one GPU
# (bench.py --rehearse-shard), native and Python exchange, with a kernel trace of the
# N = 8 step (tools/step_trace.py); optional test files first (TESTS=...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4shard
rm -rf $OUT; mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
fi
# VARIANTS: N:exchange[:VAR=value]
for v in ${VARIANTS:-8:native 8:python 4:native 2:native}; do
  IFS=: read -r n x e <<< "$v"
  tag=${n}_${x}${e:+_${e//=/}}
  timeout -k 10 300 env $e python -u bench.py --rehearse-shard $n --exchange $x --steps ${STEPS:-200} --warmup 5 > $OUT/shard$tag.json 2> $OUT/shard$tag.err || { tail -5 $OUT/shard$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/shard$tag.json')); print('$v', d['rehearsal']['step_us'], 'host', d['host_enqueue_us_per_step'], d['kernels'], d['dist'] and d['dist'].get('consistent'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --rehearse-shard 8 --steps 200 --warmup 5 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 tools/step_trace.py $OUT/trace --skip 60 --show 2 | tee $OUT/step_trace.txt
