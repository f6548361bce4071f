set -u
OUT=gpurun_out/c4chunk; mkdir -p $OUT
for r in 1 2; do for v in head onechunk; do
  timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --no-cpu-baseline --lib tools/ab_libs/$v.so > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail -5 $OUT/${v}_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', '$r', round(d['ms_per_step'], 3))"
done; done
