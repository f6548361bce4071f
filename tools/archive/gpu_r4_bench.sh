#!/bin/bash
# GPU call: the default bench line (N = 1), the N = 2 gloo rehearsal (two ranks on one
# GPU) with the exchange self-check, and the same with a deliberately corrupted block.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4bench
mkdir -p $OUT
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $OUT/default.json 2> $OUT/default.err || { tail -5 $OUT/default.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/default.json')); print('default', d['value'], d['ms_per_step'], d['host_enqueue_us_per_step'], d['kernels'], d['roofline']['frac'], d['roofline'].get('frac_survey_model'), d['dist'])"
if [ "${REHEARSE:-1}" = 1 ]; then
for c in "" "--check-corrupt"; do
  timeout -k 10 400 python -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 20 --warmup 3 --no-extra $c > $OUT/g2$c.json 2> $OUT/g2$c.err || { tail -5 $OUT/g2$c.err; exit 1; }
  tail -1 $OUT/g2$c.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('g2 $c', d['value'], d['ms_per_step'], d['config']['leases_per_gpu'], d['dist']['consistent'], d['dist']['exchange_check']['blocks_hash_equal'], d['dist']['exchange_check']['sample'])"
done
fi
