#!/bin/bash
# GPU call (round 5): the N>1 evidence lines -- the N=2/4/8 shard rehearsals (one rank's
# step of an N-GPU configs[3] node on one GPU), and the N=2 gloo rehearsal of the whole
# distributed path (two ranks on cuda:0) with its exchange self-check, plain and with a
# corrupted block (the check must say consistent false).  Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5evid}
mkdir -p $OUT
for n in 8 4 2; do
  timeout -k 10 300 python -u bench.py --workload c3 --rehearse-shard $n --steps 200 --warmup 20 > $OUT/shard${n}_step.json 2> $OUT/shard${n}_step.err || { tail -5 $OUT/shard${n}_step.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/shard${n}_step.json').read().strip().splitlines()[-1])
print('shard $n', d['rehearsal']['step_us'], d['dist']['consistent'] if d.get('dist') else None)"
done
for tag in selfcheck selfcheck_corrupt; do
  extra=""; [ $tag = selfcheck_corrupt ] && extra="--check-corrupt"
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --same-device --dist-backend gloo --steps 30 --warmup 5 $extra > $OUT/g2_$tag.json 2> $OUT/g2_$tag.err || { tail -8 $OUT/g2_$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/g2_$tag.json').read().strip().splitlines()[-1])
print('g2 $tag', d['value'], d['ms_per_step'], {k: d['dist'].get(k) for k in ('consistent', 'rccl_nranks', 'step_us_min', 'step_us_max', 'ranks')})"
done
