#!/bin/bash
# GPU call: C2 timeline of the current tree; C2 large class alone and the whole tick,
# base build against a variant (VAR, default tools/variants/lib_nohalf.so); the C3
# bench line (rest kernel's host word only on change).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
B=doorman_amd/libdoorman_hip_base.so
V=${VAR:-tools/variants/lib_nohalf.so}
timeout -k 10 120 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dense or c1 or split" > gpurun_out/r3h/pytest.log 2>&1
s=$?; tail -1 gpurun_out/r3h/pytest.log; [ $s -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r3h/pytest.log | head; exit $s; }
timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/r3h/b.json 2> gpurun_out/r3h/b.err || { tail -5 gpurun_out/r3h/b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3h/b.json').read().strip().splitlines()[-1])
print('c3', round(d['ms_per_step']*1000,1), 'us/step', {k: v['avg_us'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python -u tools/large_probe.py --steps 30 $B $V $B $V > gpurun_out/r3h/probe.log 2>&1 || { tail -5 gpurun_out/r3h/probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3h/probe.log
timeout -k 10 300 python -u tools/large_probe.py --small --steps 30 $B > gpurun_out/r3h/probe_small.log 2>&1 || { tail -5 gpurun_out/r3h/probe_small.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3h/probe_small.log
timeout -k 10 400 python -u tools/ab.py --workload c2 --rounds 8 --steps 20 --per-kernel $B $V > gpurun_out/r3h/ab.log 2>&1 || { tail -5 gpurun_out/r3h/ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3h/ab.log | tail -30
bash tools/gpu_c2tl.sh > gpurun_out/r3h/tl.log 2>&1; tail -25 gpurun_out/r3h/tl.log
