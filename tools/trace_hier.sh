#!/bin/bash
# Kernel + copy trace of the hierarchical bench step (one GPU): where the exchange's time goes.
export TMPDIR=/tmp
rm -rf gpurun_out/trace_hier; mkdir -p gpurun_out/trace_hier
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_hier -o run -- \
  python3 bench.py --hier --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/trace_hier/log 2>&1
