#!/bin/bash
# Instruction mix per kernel (one --pmc pass, 8 SQ counters) + kernel-trace stats
# for a workload: is a kernel bound by VALU issue or by memory?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
OUT=gpurun_out/valu_$W
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d $OUT/pmc -o run -- python3 bench.py --steps 5 --warmup 2 --workload $W --no-cpu-baseline > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 2 --workload $W --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 tools/valu_summary.py $OUT
