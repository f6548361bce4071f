set -u
mkdir -p gpurun_out/ab_ev
for r in 1 2; do
  for v in head dev sysoff; do
    timeout -k 10 120 python -u bench.py --workload c3 --rehearse-shard 8 --steps 200 --warmup 20 --no-cpu-baseline --lib tools/ab_libs/$v.so > gpurun_out/ab_ev/s8_${v}_$r.json 2> gpurun_out/ab_ev/s8_${v}_$r.err || { tail -5 gpurun_out/ab_ev/s8_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab_ev/s8_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', '$r', round(d['ms_per_step']*1e3,2), {k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
