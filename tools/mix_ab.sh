#!/bin/bash
# Instruction mix + stall counters of the tick kernels for several library builds
# (one --pmc pass per build, 8 SQ counters):  WORKLOAD=c3 tools/mix_ab.sh LIB.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-c3}
CTRS=${CTRS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY}
for L in "$@"; do
  n=$(basename $L .so)
  OUT=gpurun_out/mix_$W/$n
  rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d $OUT -o run -- python3 tools/tick_lib.py --workload $W --steps 5 $L > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
  python3 - "$OUT" "$n" <<'PY'
import csv, glob, sys, collections
d, n = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, v in acc.items():
    disp = cnt[(k, "SQ_WAVES")] or 1
    print(n, k, " ".join(f"{c}={v[c]/disp:.4g}" for c in sorted(v)))
PY
done
