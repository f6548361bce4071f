#!/bin/bash
# GPU call (round 5, batch 3): the C2 bench line twice (in-tree build), C2 A/B of the
# empty-redo probes, then a C2 kernel timeline (rocprofv3 --kernel-trace -> tools/timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r5b3
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c2 --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { tail -5 $OUT/bench_c2_$i.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/bench_c2_$i.json').read().strip().splitlines()[-1])
print('c2 bench', d['ms_per_step'], 'enqueue us', d['host_enqueue_us_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
PAIRS="base4:rnull64 base4:rnull1" TAG=r5b3 bash tools/gpu_r5_ab.sh || exit 1
TL=gpurun_out/r5b3tl
rm -rf $TL; mkdir -p $TL
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $TL/trace -o run -- python3 bench.py --workload c2 --steps 200 --warmup 3 --no-cpu-baseline --no-extra > $TL/log.txt 2>&1 || { tail -5 $TL/log.txt; exit 1; }
python3 tools/timeline.py $TL/trace --skip 30 > $TL/timeline.txt 2>&1; tail -40 $TL/timeline.txt
