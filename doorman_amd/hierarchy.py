"""Multi-GPU orchestration: resource sharding and the intermediate-server hierarchy.

* Sharding: resources are independent (no cross-resource term in
  go/server/doorman/algorithm.go), so a node splits the resource-id range into
  contiguous shards balanced by lease count, one per GPU, and every GPU runs its
  ticks with no data-path communication.

* Hierarchy (server.go:227-323 on the intermediate, :822-901 on the root): every
  GPU is one intermediate server.  Sharded (configs[3]): each GPU
  holds its contiguous range of the resources; replicated: each GPU holds its own
  clients of the same R resources.  Per exchange each server publishes its
  request -- {SumWants, Count} per resource plus its validation flags
  (dm_publish_totals) -- one RCCL all-gather over xGMI shares them, every rank
  evaluates the root's round redundantly on its own copy of the root store,
  loads its own new templates (grant, root algorithm, or the "*" default) into
  its leaf (dm_hier_root_tick) and runs its leaf tick; pipelined, the exchange
  runs beside the next leaf tick with one tick of lag.

torch is plumbing here (device buffers and torch.distributed); import it before
doorman_amd so the HIP library binds to torch's HIP runtime.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import workloads as W


def rccl_unique_id() -> bytes:
    """dm_rccl_unique_id: a new id for the exchange's RCCL communicator (rank 0)."""
    from . import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(_lib.DM_RCCL_ID_BYTES)
    _lib.check(L.dm_rccl_unique_id(buf), None, L)
    return buf.raw


# What one writeback tick moves per lease and per resource (bench.LEASE_BYTES /
# RESOURCE_BYTES): read wants, has, int32 subclients, write gets; the
# resource's config record, running sums in and out and its state byte.
LEASE_COST_B = 28.0
RESOURCE_COST_B = 97.0


def tick_cost(seg_sizes) -> np.ndarray:
    """Predicted cost of each resource in one tick, in bytes moved.  A tick is HBM-bound
    and its kernel classes share the HBM (profiles/r05_c2_classes.md: the C2 tick is the
    classes' shared HBM time), so bytes predict time.  Per resource, not per lease: a
    Zipf population's singletons cost 97 B of record against 28 B of row each, and a
    lease-count split leaves them all on the last shard (2.2x the mean bytes at N = 8 on
    configs[2])."""
    sizes = np.asarray(seg_sizes, dtype=np.float64)
    return LEASE_COST_B * sizes + RESOURCE_COST_B


# Tick time per byte of each size class of a resource-id shard of configs[2], fitted
# (non-negative least squares, with a fixed ~10 us per tick) to every rank's rehearsed
# step of the contiguous N = 2 / 4 / 8 shards on one MI355X (profiles/r06_c2_shard*_ranks
# _contiguous.json): a shard's classes share the GPU's workgroup slots rather than only
# its HBM, so a class that is latency-bound per byte (the tiles of 2-4-row resources
# with the sub-wave groups of the 5-6-row ones beside them) costs several times what
# the bytes say.  (upper size of the class, us per MB of tick_cost)
C2_CLASS_US_PER_MB = ((1, 0.087), (4, 0.469), (16, 0.072), (256, 0.195), (4096, 0.150), (1 << 62, 0.250))


def tick_time(seg_sizes) -> np.ndarray:
    """Predicted tick time of each resource of a shard (us): tick_cost weighted by its
    size class's measured rate (C2_CLASS_US_PER_MB)."""
    sizes = np.asarray(seg_sizes, dtype=np.int64)
    w = np.zeros(len(sizes))
    lo = 0
    for hi, us in C2_CLASS_US_PER_MB:
        w[(sizes > lo) & (sizes <= hi)] = us
        lo = hi
    return tick_cost(sizes) * w / 1e6


def partition(seg_sizes, world: int, cost=None) -> np.ndarray:
    """Contiguous resource ranges balanced by predicted tick cost (tick_cost, or the
    given per-resource cost): boundaries b[0..world] with shard k = resources
    [b[k], b[k+1]).  With one size for every resource (configs[3]) this is the even
    lease-count split."""
    sizes = np.asarray(seg_sizes, dtype=np.int64)
    R = len(sizes)
    if world <= 1 or R == 0:
        return np.array([0, R], dtype=np.int64)
    c = tick_cost(sizes) if cost is None else np.asarray(cost, dtype=np.float64)
    assert len(c) == R
    csum = np.concatenate([[0.0], np.cumsum(c)])
    total = csum[-1]
    bounds = [0]
    for k in range(1, world):
        target = total * k / world
        b = int(np.searchsorted(csum, target, side="left"))
        # pick the closer of b-1 / b, keep ranges monotone and non-empty where possible
        if b > 0 and abs(csum[b - 1] - target) <= abs(csum[min(b, R)] - target):
            b -= 1
        b = max(b, bounds[-1] + (1 if R - bounds[-1] > world - k else 0))
        if R >= world:  # leave at least one resource for each later shard
            b = min(b, R - (world - k))
        bounds.append(min(b, R))
    bounds.append(R)
    return np.asarray(bounds, dtype=np.int64)


def assign_lpt(seg_sizes, world: int, cost=None) -> np.ndarray:
    """Owner rank of every resource: longest-processing-time-first over the predicted
    tick cost (tick_cost), i.e. each resource, costliest first, to the rank with the
    least cost so far.  Unlike contiguous ranges every rank then holds the same mix of
    size classes -- a shard of a Zipf population's tail is all tiles, of its head all
    large chain, and the classes' kernels run at different rates per byte (the N = 8
    contiguous shards of configs[2] measured 12-30 us per tick at equal bytes,
    profiles/r06_c2_shard8_ranks_contiguous.json) -- and the largest resources spread
    over the ranks first."""
    import heapq
    sizes = np.asarray(seg_sizes, dtype=np.int64)
    c = tick_cost(sizes) if cost is None else np.asarray(cost, dtype=np.float64)
    owner = np.zeros(len(sizes), dtype=np.int32)
    if world <= 1:
        return owner
    heap = [(0.0, k) for k in range(world)]
    for i in np.argsort(-c, kind="stable"):
        load, k = heapq.heappop(heap)
        owner[i] = k
        heapq.heappush(heap, (load + float(c[i]), k))
    return owner


# The size classes of a tick: tiles, the sub-wave launch, the four
# workgroup bins, the large chain.  (first, last row count)
SIZE_CLASSES = ((1, 4), (5, 256), (257, 512), (513, 1024), (1025, 2048), (2049, 4096), (4097, 1 << 62))


def assign_by_class(seg_sizes, world: int, cost=None) -> np.ndarray:
    """Owner rank of every resource, balanced class by class: within each size class
    (SIZE_CLASSES, the largest first) longest-processing-time-first over tick_cost from
    empty ranks, so every rank runs every class the store has with 1/N of its work (a
    global LPT leaves the rank that took the largest resource without whole classes,
    and a shard's tick is set by the classes it runs -- each a latency-bound launch at
    a shard's size -- as much as by its bytes: profiles/r06_c2_shard8_ranks_lpt.json);
    then the smallest resources (the tiles' class, 125 B each) move from ranks above
    the mean predicted bytes to ranks below it, so the bytes balance too (the one
    resource larger than a rank's share of its class, configs[2]'s 1M-row head, stays
    on its rank)."""
    import heapq
    sizes = np.asarray(seg_sizes, dtype=np.int64)
    c = tick_cost(sizes) if cost is None else np.asarray(cost, dtype=np.float64)
    owner = np.zeros(len(sizes), dtype=np.int32)
    if world <= 1:
        return owner
    for lo, hi in SIZE_CLASSES[::-1]:
        ids = np.flatnonzero((sizes >= lo) & (sizes <= hi))
        heap = [(0.0, k) for k in range(world)]
        for i in ids[np.argsort(-c[ids], kind="stable")]:
            load, k = heapq.heappop(heap)
            owner[i] = k
            heapq.heappush(heap, (load + float(c[i]), k))
    load = np.bincount(owner, weights=c, minlength=world)
    target = load.mean()
    small = np.flatnonzero(sizes <= SIZE_CLASSES[0][1])[::-1]  # the smallest first (the Zipf tail's end)
    for k in np.argsort(-load):
        if load[k] <= target:
            break
        for r in small[owner[small] == k]:
            if load[k] <= target * 1.002:
                break
            d = int(np.argmin(load))
            if load[d] + c[r] > target:
                break
            owner[r] = d
            load[k] -= c[r]
            load[d] += c[r]
    return owner


def shard(snap: dict, world: int, rank: int, cost=None) -> dict:
    """This rank's contiguous range of the snapshot's resources (partition)."""
    b = partition(np.diff(snap["seg_off"]), world, cost)
    return W.subset_range(snap, int(b[rank]), int(b[rank + 1]))


def root_snapshot(n_resources: int, n_servers: int, kind, capacity, lease_length_s=20, refresh_interval_s=5) -> dict:
    """The root server's store for the hierarchy: R resources x G server rows
    (replicated layout; n_servers = 1 for the sharded layout's one row per
    resource), all released until the first exchange (dm_hier_root_tick)."""
    G = n_servers
    N = n_resources * G
    return W.make_snapshot(np.full(n_resources, G), np.zeros(N), np.zeros(N), np.zeros(N, np.int64),
                           np.full(N, W.RELEASED), kind, capacity, lease_length_s, refresh_interval_s,
                           aggregates=True)


class HierarchicalTick:
    """One rank of the hierarchy: an intermediate server (leaf engine) plus a
    redundant copy of the root (root engine), both on this rank's GPU.

    Layouts (dm_hier_layout): shard_lo None -- replicated, every server holds all
    n_resources resources (root store R x G rows); shard_lo = G + 1 bounds -- sharded
    by resource id, server g holds resources [shard_lo[g], shard_lo[g+1]) and its leaf
    only those (root store R rows, one per resource).

    gather(src, dst): all-gather of every server's published block ([stride, 2]
    float64: record 0 = the request's validation flags, 1 + i = {SumWants, Count} of
    its i-th resource) into dst [G * stride, 2] in server order
    (torch.distributed.all_gather_into_tensor over RCCL on a node; a local copy in
    single-process tests).

    pipelined: the exchange (publish -> all-gather -> root round) runs on a stream of
    its own beside the next leaf tick, and each leaf tick takes the templates of the
    exchange enqueued before the previous tick (dm_hier_pipeline: one tick of lag, as
    the reference's intermediate refreshes upstream on its own loop, server.go:227-323).
    Otherwise every tick first runs its exchange, stream-ordered on one stream."""

    def __init__(self, torch, leaf, root, n_resources: int, n_servers: int, server: int, gather, shard_lo=None,
                 pipelined: bool = False, native: str | None = None, comm_id: bytes | None = None,
                 lag: int | None = None, comm_ranks: int | None = None):
        """native: the whole pipelined step in one library call (dm_hier_step) instead of
        the Python sequence below -- "rccl": the blocks gathered by the library's own RCCL
        communicator (comm_id: rank 0's dm_rccl_unique_id, the same bytes on every rank;
        dm_hier_comm_init is collective), "local": without a collective (one server, or one
        rank's rehearsal: its block copied into its slot of `gather`-less gathered buffer)."""
        from . import _lib
        self.torch = torch
        self.leaf, self.root = leaf, root
        self.R, self.G, self.g = n_resources, n_servers, server
        self.gather = gather
        self.native = native
        if native is not None:
            assert native in ("rccl", "local") and pipelined, "dm_hier_step is the pipelined step"
        self.pipelined = pipelined
        L = root._L
        if shard_lo is None:
            self.stride = 1 + self.R
            _lib.check(L.dm_hier_layout(root._ctx, self.G, None, self.stride), root._ctx, L)
        else:
            lo = np.ascontiguousarray(shard_lo, dtype=np.int64)
            assert len(lo) == self.G + 1 and lo[0] == 0 and lo[-1] == self.R
            self.stride = 1 + int(np.diff(lo).max())
            _lib.check(L.dm_hier_layout(root._ctx, self.G, lo.ctypes.data, self.stride), root._ctx, L)
        dev = torch.device("cuda", torch.cuda.current_device())
        # pipelined: the leaf's writeback ticks publish their blocks themselves
        # (dm_publish_ring, a ring of three: an exchange may still read the block of
        # the tick before the previous one); otherwise one block published before
        # each exchange (dm_publish_totals)
        nbuf = 3 if pipelined else 1
        self.totals = [torch.zeros((self.stride, 2), dtype=torch.float64, device=dev) for _ in range(nbuf)]
        # one server: the all-gather is the identity, so the root reads the block in place.
        # The exchange stream runs gather -> root round in order, so one gathered buffer
        # serves every step.
        g1 = torch.zeros((self.G * self.stride, 2), dtype=torch.float64, device=dev) if self.G > 1 else None
        self.gathered = self.totals if self.G == 1 else [g1] * nbuf
        self.step = 0
        # The library's kernels and torch's collective share streams of their own:
        # torch's default stream is the HIP null stream, which dm_set_stream cannot
        # select (NULL restores the context's own stream) and which does not order the
        # library's non-blocking streams.  Unpipelined: one stream, so publish ->
        # all-gather -> root -> templates -> leaf tick are ordered without host syncs.
        # Pipelined with G > 1, the exchange (all-gather + root round) gets a stream of its
        # own so the collective overlaps the next leaf tick.  With one server there is no
        # collective and the root round (~10 us) is cheaper than the two cross-queue hops
        # a second stream costs per step (~20 us of idle GPU each): the
        # exchange then runs on the leaf's stream, still one tick of lag (staged slots).
        self.stream = torch.cuda.Stream(device=dev)
        own = self.G > 1
        # the exchange's kernels (gather, root round) are few and short, but beside a leaf tick
        # that fills every CU they wait for slots: a high-priority queue lets them in first
        self.xstream = torch.cuda.Stream(device=dev, priority=-1) if pipelined and own else self.stream
        # the buffers above are zeroed on torch's current stream: the library's streams
        # (which dm_publish_ring's flag reset and every later write run on) wait for that
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        if self.xstream is not self.stream:
            self.xstream.wait_stream(cur)
        leaf.set_stream(self.stream.cuda_stream)
        root.set_stream(self.xstream.cuda_stream)
        # lag: ticks of lag of the pipelined templates (dm_hier_pipeline): default 1 with the
        # exchange on the leaf's stream, 2 with a stream of its own (the exchange then has a
        # whole tick to finish before the leaf takes its templates: the leaf never waits)
        if lag is None:
            lag = 2 if self.xstream is not self.stream else 1
        self.lag = lag if pipelined else 0
        _lib.check(leaf._L.dm_hier_pipeline(leaf._ctx, self.lag), leaf._ctx, leaf._L)
        ring = (ctypes.c_void_p * nbuf)(*[t.data_ptr() for t in self.totals])
        if native is None:
            _lib.check(leaf._L.dm_publish_ring(leaf._ctx, nbuf if pipelined else 0, ring), leaf._ctx, leaf._L)
            return
        if native == "rccl":
            assert comm_id is not None and len(comm_id) == _lib.DM_RCCL_ID_BYTES
            idb = ctypes.create_string_buffer(bytes(comm_id), _lib.DM_RCCL_ID_BYTES)
            nr = self.G if comm_ranks is None else comm_ranks  # (tests: a one-rank communicator on one GPU)
            _lib.check(L.dm_hier_comm_init(root._ctx, idb, nr, self.g if nr == self.G else 0), root._ctx, L)
        gp = self.gathered[0].data_ptr() if self.G > 1 else None
        _lib.check(L.dm_hier_attach(leaf._ctx, root._ctx, self.g, ring, nbuf, gp, self.xstream.cuda_stream),
                   root._ctx, L)

    def comm_info(self):
        """(ranks, rank) as the library's RCCL communicator itself reports them
        (dm_hier_comm_info: ncclCommCount / ncclCommUserRank), or None without one."""
        from . import _lib
        if self.native != "rccl":
            return None
        L = self.root._L
        n, r = ctypes.c_int(0), ctypes.c_int(-1)
        _lib.check(L.dm_hier_comm_info(self.root._ctx, ctypes.byref(n), ctypes.byref(r)), self.root._ctx, L)
        return n.value, r.value

    def exchange(self, now_ns: int):
        """publish -> all-gather -> the root's round -> this server's new templates
        (pipelined: the block the last leaf tick published)."""
        from . import _lib
        k = self.step % len(self.totals)
        self.step += 1
        totals, gathered = self.totals[k], self.gathered[k]
        if not self.pipelined:
            self.leaf.publish_totals(totals.data_ptr())
        else:  # the exchange stream after the leaf tick that published the block
            self.leaf.stream_wait(self.xstream.cuda_stream)
        if self.G > 1:
            with self.torch.cuda.stream(self.xstream):  # the collective orders with the exchange stream
                self.gather(totals, gathered)
        L = self.root._L
        _lib.check(L.dm_hier_root_tick(self.root._ctx, gathered.data_ptr(), self.G, int(now_ns),
                                       self.leaf._ctx, self.g), self.root._ctx, L)

    def status(self) -> np.ndarray:
        """dm_hier_status: per-server flags of the last exchange (0 = request accepted)."""
        from . import _lib
        st = np.zeros(self.G, np.uint32)
        _lib.check(self.root._L.dm_hier_status(self.root._ctx, st.ctypes.data, self.G), self.root._ctx, self.root._L)
        return st

    def check(self):
        """Raise DmError(DM_E_ARGUMENT) if the root rejected some server's request in the
        last exchange (a band with num_clients < 1, server.go:863-866, or a Count beyond
        2^31): the reference fails that server's GetServerCapacity RPC."""
        from . import _lib
        st = self.status()
        bad = np.flatnonzero(st)
        if len(bad):
            raise _lib.DmError(_lib.DM_E_ARGUMENT, f"root rejected the requests of servers {bad.tolist()} "
                                                   f"(flags {st[bad].tolist()}: 1 = num_clients < 1, 2 = Count >= 2^31)")

    def tick(self, now_ns: int, asynchronous: bool = False):
        if self.native is not None:  # the leaf tick + the exchange in one library call
            from . import _lib
            self.step += 1
            _lib.check(self.root._L.dm_hier_step(self.leaf._ctx, self.root._ctx, int(now_ns)), self.root._ctx,
                       self.root._L)
            if not asynchronous:
                self.sync()
            return
        if self.pipelined:  # the tick (templates staged one exchange ago; it publishes its block), then
            # this step's exchange of that block
            self.leaf.apportion(now_ns, writeback=True, asynchronous=True)
            self.exchange(now_ns)
            if not asynchronous:
                self.sync()
        else:
            self.exchange(now_ns)
            self.leaf.apportion(now_ns, writeback=True, asynchronous=asynchronous)

    def sync(self):
        self.stream.synchronize()
        self.xstream.synchronize()
        self.leaf.sync()
        self.root.sync()
