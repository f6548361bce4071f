#!/bin/bash
# GPU call: FETCH_SIZE / WRITE_SIZE / SQ instruction counts of the dense tick kernel for
# tools/c4_variants.py variants (one process per variant and pass), then a per-variant
# summary.  Every step has its own limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c4pmc}
rm -rf $OUT; mkdir -p $OUT
for v in ${VARIANTS:-fs_free ps_free}; do
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
    tag=$v-$(echo $pass | cut -d' ' -f1)
    WARM=50 timeout -k 10 240 rocprofv3 --pmc $pass --output-format csv -d $OUT/$tag -o run -- \
      python3 tools/c4_variants.py 10 $v > $OUT/$tag.log 2>&1 || { echo "STOP $tag"; tail -5 $OUT/$tag.log; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
d = sys.argv[1]
for sub in sorted(os.listdir(d)):
    f = glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    acc = {}
    for row in csv.DictReader(open(f[0])):
        if "k_block_dense" not in row["Kernel_Name"]:
            continue
        acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    print(sub, {k: round(sum(v) / len(v)) for k, v in acc.items()}, "dispatches", len(next(iter(acc.values()), [])))
PY
