#!/bin/bash
# round 3: default bench + rocprof kernel trace of it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-extra > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
s=$?; python -c "
import json; d=json.loads(open('gpurun_out/bench_c3.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], d['kernels'])"; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_c3.err; exit $s; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu-baseline --no-extra > $GRAFT_REPO_ROOT/gpurun_out/prof_c3.log 2>&1
s=$?; cd $GRAFT_REPO_ROOT; find gpurun_out/prof_c3 -name "*stats*" | head; exit $s
