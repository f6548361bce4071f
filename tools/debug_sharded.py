"""Debug: the sharded exchange of tests/test_hierarchy_gpu.py, step 0, printed."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import test_hierarchy_gpu as T
from doorman_amd import workloads as W, _lib
from doorman_amd.engine import Engine
from doorman_amd.hierarchy import partition, root_snapshot
import hier_model as M
NOW = W.NOW_NS
L = _lib.lib()
G = 3
rng = np.random.default_rng(31)
sizes = rng.integers(5, 700, 60)
R = len(sizes)
lo = partition(sizes, G)
S = 1 + int(np.diff(lo).max())
print("lo", lo, "S", S)
rcfg = T.root_config(R, rng)
full = W.make_snapshot(sizes, rng.uniform(0.2, 3.0, int(sizes.sum())) * 1000.0 / np.repeat(sizes, sizes),
                       0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
leaves, roots = [], []
for g in range(G):
    shard = W.subset(full, np.arange(lo[g], lo[g + 1]))
    e = Engine(0)
    e.load(M.with_config(shard, M.default_config(int(lo[g + 1] - lo[g]))))
    leaves.append(e)
    root = Engine(0)
    root.load(M.with_config(root_snapshot(R, 1, W.FAIR_SHARE, 1.0), rcfg))
    _lib.check(L.dm_hier_layout(root._ctx, G, lo.ctypes.data, S), root._ctx)
    roots.append(root)
gathered = torch.zeros((G * S, 2), dtype=torch.float64, device="cuda")
for g in range(G):
    leaves[g].publish_totals(gathered[g * S:(g + 1) * S].data_ptr())
    leaves[g].sync()
rec = gathered.cpu().numpy()
for g in range(G):
    print("server", g, "flags", rec[g * S, 0:1].view(np.int64), "first recs", rec[g * S + 1:g * S + 4, 0])
for g in range(G):
    _lib.check(L.dm_hier_root_tick(roots[g]._ctx, gathered.data_ptr(), G, NOW, leaves[g]._ctx, g), roots[g]._ctx)
    roots[g].sync()
st = np.zeros(G, np.uint32)
print("status", L.dm_hier_status(roots[0]._ctx, st.ctypes.data, G), st)
s0 = roots[0].read_store()
print("has", np.round(s0["has"], 2))
print("wants", np.round(s0["wants"], 2))
print("sub", s0["subclients"])
print("kind", rcfg["kind"])
