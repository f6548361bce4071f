#!/bin/bash
# GPU call: C2's large resources alone, chain vs the persistent path over grid /
# ticket-batch settings (tools/large_probe.py), then the full C2 tick A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=doorman_amd/libdoorman_hip.so
V=${VARIANTS:-"$L@DM_LARGE_PATH=0 $L@DM_LARGE_PATH=2,DM_FLOW_WG=2,DM_FLOW_BATCH=1 $L@DM_LARGE_PATH=2,DM_FLOW_WG=2,DM_FLOW_BATCH=4 $L@DM_LARGE_PATH=2,DM_FLOW_WG=4,DM_FLOW_BATCH=4 $L@DM_LARGE_PATH=2,DM_FLOW_WG=4,DM_FLOW_BATCH=16 $L@DM_LARGE_PATH=2,DM_FLOW_WG=1,DM_FLOW_BATCH=4"}
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $V > gpurun_out/flow_sweep.log 2>&1
s=$?; cat gpurun_out/flow_sweep.log | grep -v amdgpu.ids; [ $s -ne 0 ] && exit $s
if [ -n "${AB:-}" ]; then
timeout -k 10 400 python -u tools/ab.py --workload c2 --rounds ${ROUNDS:-6} --steps 20 --per-kernel $AB > gpurun_out/ab_flow.log 2>&1
s=$?; grep -v amdgpu.ids gpurun_out/ab_flow.log | tail -20; exit $s
fi
