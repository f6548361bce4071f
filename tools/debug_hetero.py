import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import numpy as np
from parity_util import *
from oracle import oracle as O
from doorman_amd import workloads as W
from doorman_amd.engine import Engine
rng = np.random.default_rng(1000)
sizes = binned_sizes(rng)
snap = snapshot_with_sizes(rng, sizes, hetero=True, edge=False)
ref = O.apportion(snap, W.NOW_NS)
e = Engine(0); e.load(snap); e.apportion(W.NOW_NS); g, x = e.leases()
ok = float_close(g, ref['gets'], row_capacity(snap))
so = snap['seg_off']
bad = np.flatnonzero(~ok)
res = np.searchsorted(so, bad, side='right') - 1
for r in np.unique(res):
    rows = bad[res == r]
    i = rows - so[r]
    print('resource', r, 'size', sizes[r], 'kind', snap['kind'][r], 'nbad', len(rows),
          'k hist', np.bincount(i // 256).tolist(), 'sub hist', np.bincount(snap['subclients'][rows]).tolist(),
          'got uniq', np.unique(g[rows])[:5])
