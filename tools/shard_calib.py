"""Calibrate configs[2]'s contiguous partition on measured per-rank ticks.

Each rehearsal (bench.py --workload c2 --rehearse-shard N --rehearse-rank -1
--c2-partition contiguous) gives every rank's step time t_k over its range
[b_k, b_k+1) of resources.  With a fixed per-tick cost F, (t_k - F) / bytes_k is the
marginal time per byte in that range; the finest rehearsal's ranges (largest N) give a
piecewise-constant density over the resource index, which the next partition weights
the bytes model with.  Prints the band table for doorman_amd/hierarchy.py.
usage: python tools/shard_calib.py F rehearsal.json [rehearsal.json ...]"""
import json
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from doorman_amd import hierarchy as H  # noqa: E402
from doorman_amd import workloads as W  # noqa: E402

F = float(sys.argv[1])
sizes = W.zipf_sizes()
byt = H.tick_cost(sizes)
dens = np.zeros(len(sizes))
cnt = np.zeros(len(sizes))
for path in sys.argv[2:]:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    b = d["bounds"]
    w = np.asarray(H.c2_time_weight(sizes)) if "weighted" in d.get("partition_note", "") else np.ones(len(sizes))
    for r in d["ranks"]:
        lo, hi = b[r["rank"]], b[r["rank"] + 1]
        dens[lo:hi] += max(r["step_us"] - F, 1.0) / (byt[lo:hi] * w[lo:hi]).sum() * w[lo:hi] * len(b)
        cnt[lo:hi] += len(b)
dens /= cnt
print(json.dumps({"F": F, "density_by_size": {int(n): float(dens[sizes == n].mean()) for n in
                                                (1, 2, 3, 4, 5, 6, 8, 12, 16, 24, 32, 64, 128, 256, 512, 1024, 2048,
                                                 4096, 8192, 100000, 1000000)}}))
