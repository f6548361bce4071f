set -u
OUT=gpurun_out/r6s8x3; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --rehearse-shard 8 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/s8_$r.json 2> $OUT/s8_$r.err || { tail -5 $OUT/s8_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/s8_$r.json').read().strip().splitlines()[-1]); print('$r', round(d['ms_per_step']*1e3, 2), d.get('host_enqueue_us_per_step'), {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
