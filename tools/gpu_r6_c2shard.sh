#!/bin/bash
# GPU call (round 6): configs[2] sharded -- every rank's step of an N-GPU node rehearsed
# one after another on this GPU (N = 2, 4, 8), then the world-size-2 gloo parity test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6c2shard}
mkdir -p $OUT
for n in ${NS:-2 4 8}; do
  timeout -k 10 300 python -u bench.py --workload c2 --rehearse-shard $n --rehearse-rank -1 --steps ${STEPS:-200} --warmup 20 \
    --c2-partition ${PART:-lpt} > $OUT/c2_shard${n}_ranks.json 2> $OUT/c2_shard${n}.err || { tail -8 $OUT/c2_shard${n}.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/c2_shard${n}_ranks.json').read().strip().splitlines()[-1])
print('c2 shard $n ${PART:-lpt}', d['step_max_over_min'], d['predicted_bytes_max_over_mean'], [r['step_us'] for r in d['ranks']])"
done
if [ "${TEST:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_c2_sharded_gpu.py \
    > $OUT/test_c2_sharded.txt 2>&1 || { tail -30 $OUT/test_c2_sharded.txt; exit 1; }
  tail -3 $OUT/test_c2_sharded.txt
fi
