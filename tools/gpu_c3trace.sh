#!/bin/bash
# GPU call: kernel trace of the default C3 step (every dispatch, blits included).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c3t
export TMPDIR=/tmp
rm -rf gpurun_out/c3t/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3t/trace -o run -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-extra ${ARGS:-} > gpurun_out/c3t/log.txt 2>&1 || { tail -5 gpurun_out/c3t/log.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/c3t/trace/**/*kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][-34:], r['Queue_Id']) for r in rows)
i0 = len(ks) - 40
t0 = ks[i0][0]
for s, e, n, q in ks[i0:]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q={q} {n}")
PY
