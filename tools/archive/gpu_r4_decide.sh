#!/bin/bash
# GPU call: per-kernel times of dm_decide's fast path on the 100k x 100k round.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r4decide
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u -m pytest -x -q -s tests/test_server_gpu.py -k "100k" > $OUT/log.txt 2>&1
s=$?
grep -E "device time|passed|failed" $OUT/log.txt | tail -3
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(f\"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e3:10.1f} us  avg {float(r['AverageNs'])/1e3:9.1f}\")
"
exit $s
