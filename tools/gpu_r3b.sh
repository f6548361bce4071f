#!/bin/bash
# round 3: new parity tests, hierarchy tests, then the default bench and the two-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_hierarchy_gpu.py tests/test_hierarchy_dist_gpu.py "tests/test_parity_gpu.py::test_c4_loop_store_apply_matches_oracle" "tests/test_parity_gpu.py::test_configs0_through_the_hip_path" "tests/test_parity_gpu.py::test_c4_full_size_properties_after_bench_rounds" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
s=$?; grep -E "passed|failed|error" gpurun_out/pytest_r3b.log | tail -3; [ $s -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/pytest_r3b.log | head -40; exit $s; }
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
s=$?; tail -c 3000 gpurun_out/bench_c3.json; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_c3.err; exit $s; }
timeout -k 10 400 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err
s=$?; tail -c 2000 gpurun_out/bench_g2.json; [ $s -ne 0 ] && { tail -20 gpurun_out/bench_g2.err; exit $s; }
exit 0
