#!/bin/bash
# SQ wave-state counters per kernel (one --pmc pass, 8 SQ counters) for a workload:
# where wave time goes (parked on waitcnt/barrier, issue-stalled, issuing VALU/LDS/VMEM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${WORKLOAD:-c2}
OUT=gpurun_out/sq_$W
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES \
  --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 2 --workload $W --no-cpu-baseline > $OUT/log 2>&1
