#!/bin/bash
# C2 kernel timeline (rocprofv3 kernel trace -> tools/timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c2tl
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload c2 --steps 200 --warmup 3 --no-cpu-baseline --no-extra > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
python3 tools/timeline.py $OUT/trace --skip 30 | tee $OUT/timeline.txt
