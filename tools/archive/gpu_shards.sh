#!/bin/bash
# GPU call: the leaf tick at configs[3]'s per-GPU shard sizes (100M leases over N = 1, 2,
# 4, 8 GPUs: 100k / 50k / 25k / 12.5k resources x 1000 clients), no exchange.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shards
export TMPDIR=/tmp
L=doorman_amd/libdoorman_hip.so
for r in 100000 50000 25000 12500; do
  timeout -k 10 300 python -u tools/ab.py --workload u${r}x1000 --rounds 4 --steps 40 --per-kernel $L > gpurun_out/shards/u$r.log 2>&1 || { tail -5 gpurun_out/shards/u$r.log; exit 1; }
  echo "R=$r"; grep -v amdgpu.ids gpurun_out/shards/u$r.log | tail -2
done
