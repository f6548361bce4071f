"""Debug: the pipelined sharded exchange of tests/test_hierarchy_gpu.py, per step."""
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
rng = np.random.default_rng(32)
sizes = rng.integers(5, 700, 60)
R = len(sizes)
lo = partition(sizes, G)
S = 1 + int(np.diff(lo).max())
rcfg = T.root_config(R, rng)
full = W.make_snapshot(sizes, rng.uniform(0.2, 3.0, int(sizes.sum())) * 1000.0 / np.repeat(sizes, sizes),
                       0.0, 1, NOW + 60 * W.NS, W.FAIR_SHARE, 1000.0)
leaves, roots = [], []
for g in range(G):
    shard = W.subset(full, np.arange(lo[g], lo[g + 1]))
    e = Engine(0)
    e.load(M.with_config(shard, M.default_config(int(lo[g + 1] - lo[g]))))
    _lib.check(L.dm_hier_pipeline(e._ctx, 1), e._ctx)
    leaves.append(e)
    root = Engine(0)
    root.load(M.with_config(root_snapshot(R, 1, W.FAIR_SHARE, 1.0), rcfg))
    _lib.check(L.dm_hier_layout(root._ctx, G, lo.ctypes.data, S), root._ctx)
    roots.append(root)
model = M.Root(rcfg, G)
gathered = torch.zeros((G * S, 2), dtype=torch.float64, device="cuda")
for t, now in enumerate([NOW, NOW + 5 * W.NS, NOW + 9 * W.NS, NOW + 30 * W.NS]):
    for g in range(G):
        leaves[g].apportion(now, writeback=True)
    for g in range(G):
        leaves[g].publish_totals(gathered[g * S:(g + 1) * S].data_ptr())
        leaves[g].sync()
    bl = T.published(gathered, G, S - 1, S)
    reqs = []
    for g in range(G):
        n = int(lo[g + 1] - lo[g])
        req = M.server_request(bl[g][0][:n], bl[g][1][:n])
        reqs.append(None if req is None else {int(lo[g]) + r: v for r, v in req.items()})
        print("step", t, "server", g, "flags", bl[g][2], "nreq", None if req is None else len(req))
    resp = model.round(now, reqs)
    for g in range(G):
        _lib.check(L.dm_hier_root_tick(roots[g]._ctx, gathered.data_ptr(), G, now, leaves[g]._ctx, g), roots[g]._ctx)
    for e in roots + leaves:
        e.sync()
    st = np.zeros(G, np.uint32)
    L.dm_hier_status(roots[0]._ctx, st.ctypes.data, G)
    rows = T._shard_rows(model, lo, R)
    d = roots[0].read_store()
    print("step", t, "status", st, "device has[:8]", np.round(d["has"][:8], 1), "model", np.round(rows["has"][:8], 1))
    print("   dev exp[:4]", d["expiry_ns"][:4] - NOW, "model", rows["expiry_ns"][:4] - NOW)
