#!/bin/bash
# GPU call: large-resource + parity tests, then C2's large class alone and the full
# C2 tick, interleaved A/B of a base build against the current one (+ flow variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_large_gpu.py tests/test_general_gpu.py "tests/test_parity_gpu.py::test_c2_zipf_full_size_sampled" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
s=$?; tail -2 gpurun_out/pytest_chain.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_chain.log | head -30; exit $s; }
B=doorman_amd/libdoorman_hip_base.so
L=doorman_amd/libdoorman_hip.so
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $B $L $B $L ${EXTRA:-} > gpurun_out/chain_probe.log 2>&1
s=$?; grep -v amdgpu.ids gpurun_out/chain_probe.log; [ $s -ne 0 ] && exit $s
timeout -k 10 400 python -u tools/ab.py --workload c2 --rounds ${ROUNDS:-8} --steps 20 $B $L > gpurun_out/ab_chain.log 2>&1
s=$?; grep -v amdgpu.ids gpurun_out/ab_chain.log | tail -6; exit $s
