#!/bin/bash
# GPU call: dense-form tests, the whole GPU suite, then C3 / C1 / u12500 / C2 ticks,
# base build against the current one (tools/ab.py, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dense
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dense/pytest.log 2>&1
s=$?; tail -1 gpurun_out/dense/pytest.log; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/dense/pytest.log | head -30; exit $s; }
B=doorman_amd/libdoorman_hip_base.so
L=doorman_amd/libdoorman_hip.so
for w in u100000x1000 c1 u12500x1000 c2; do
  timeout -k 10 300 python -u tools/ab.py --workload $w --rounds 6 --steps 30 --per-kernel $B $L > gpurun_out/dense/ab_$w.log 2>&1 || { tail -5 gpurun_out/dense/ab_$w.log; exit 1; }
  echo "== $w"; grep -v amdgpu.ids gpurun_out/dense/ab_$w.log | grep -E "tick med"
done
