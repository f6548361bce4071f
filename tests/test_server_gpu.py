"""The round-oriented GetCapacity dispatch (dm_server_*, doorman_amd/server.py) on
the GPU, against the reference's server tests and a model of the reference
server (store.go Clean/Release/Assign, resource.go Decide) whose rounds the CPU
oracle decides on the same snapshots.

Bar: expiry times and refresh intervals exact; capacities within
1e-9 * max(|ref|, capacity).
"""
import json
import os

import numpy as np
import pytest

from doorman_amd import workloads as W
from oracle import oracle as O
from parity_util import float_close

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "reference_kats.json")))
NOW = W.NOW_NS
I64_MIN, I64_MAX = np.iinfo(np.int64).min, np.iinfo(np.int64).max


def _server(resources, slots=4):
    from doorman_amd.server import TickServer
    return TickServer(resources, slots=slots)


def _learning_end(case, started_at):
    lmd = case["learning_mode_duration"]
    dur = case["lease_length"] if lmd is None else lmd  # resource.go:157-161
    return started_at + dur * W.NS if dur > 0 else 0   # server.go:173-179


def _res_cfg(case, started_at):
    return {"kind": case["kind"], "capacity": case["capacity"], "lease_length_s": case["lease_length"],
            "refresh_interval_s": case["refresh_interval"], "learning_end_ns": _learning_end(case, started_at)}


def test_learning_mode_kat():
    """server_test.go:339-382: in learning mode a client gets what it reports having
    (20, then 90); a resource created after the learning period decides (100)."""
    case = next(c for c in KATS["server"] if c["name"] == "TestLearningMode")
    master_at = NOW - W.NS // 2
    resources = {"res": _res_cfg(case, master_at)}
    later = [s for s in case["steps"] if s.get("new_resource")]
    for k, s in enumerate(later):
        resources[f"res{k}"] = _res_cfg(case, NOW - s["age_s"] * W.NS)
    srv = _server(resources)
    k_new = 0
    for step in case["steps"]:
        res = "res"
        if step.get("new_resource"):
            res, k_new = f"res{k_new}", k_new + 1
        t = srv.get_capacity("client", res, step["has"], step["wants"])
        srv.tick(NOW)
        lease = srv.lease(t)
        assert lease.capacity == step["gets"]
        assert lease.refresh_interval == case["refresh_interval"]
        assert lease.expiry_time == (NOW + case["lease_length"] * W.NS) // W.NS
    srv.close()


def test_get_server_capacity_bands_kat():
    """server_test.go:505-553: the bands of a GetServerCapacity become one request
    (sum of wants, sum of num_clients) that FairShare grants 100."""
    case = next(c for c in KATS["server"] if c["name"] == "TestGetServerCapacity")
    wants, sub = O.aggregate_bands([b[0] for b in case["bands"]], [b[1] for b in case["bands"]])
    srv = _server({"res": _res_cfg(case, NOW - W.NS)})
    t = srv.get_capacity("server-1", "res", case["has"], wants, sub)
    srv.tick(NOW)
    assert srv.lease(t).capacity == case["gets"]
    srv.close()


def test_wrong_number_of_clients_is_invalid_argument():
    """server_test.go:483-503: num_clients < 1 is codes.InvalidArgument."""
    from doorman_amd._lib import DM_E_ARGUMENT, DM_E_RANGE
    from doorman_amd.server import ServerError
    srv = _server({"res": {"kind": W.PROPORTIONAL_SHARE, "capacity": 100.0}})
    with pytest.raises(ServerError) as e:
        srv.get_capacity("c", "res", 0.0, 10.0, 0)
    assert e.value.code == DM_E_ARGUMENT
    with pytest.raises(ServerError) as e:
        srv.get_capacity("c", "no-such-resource", 0.0, 10.0, 1)
    assert e.value.code == DM_E_RANGE
    srv.release_capacity("c", "no-such-resource")  # ignored, like server.go:706-710
    srv.close()


class ServerModel:
    """The reference server (test infrastructure): one LeaseStore per resource (the
    oracle's restatement of store.go).  A round: Clean, the ReleaseCapacity calls,
    then every request's Resource.Decide (resource.go:100-113, ending with its
    Assign, store.go:153-167) in queue order on the live store, as res.mu serialises
    the reference's GetCapacity calls (resource.go:103-104)."""

    def __init__(self, resources):
        self.ids = list(resources)
        self.cfg = resources
        self.cid = {}
        self.stores = {r: O.Store(256) for r in self.ids}
        self.tab = {r: O.make_cfg(1, kind=c["kind"], capacity=c["capacity"], lease_length_s=c.get("lease_length_s", 300),
                                  refresh_interval_s=c.get("refresh_interval_s", 5),
                                  learning_end_ns=c.get("learning_end_ns", I64_MIN),
                                  parent_expiry_ns=c.get("parent_expiry_ns", I64_MAX),
                                  safe_capacity=c.get("safe_capacity", np.nan))[0] for r, c in resources.items()}

    def _id(self, c):
        return self.cid.setdefault(c, len(self.cid))

    def clients(self, r):
        return sum(self.stores[r].has_client(i) for i in self.cid.values())

    def round(self, now, requests, releases):
        for r in self.ids:
            self.stores[r].clean(now)  # store.go:169-181
        for c, r in releases:  # server.go:705-711
            if c in self.cid:
                self.stores[r].release(self.cid[c])
        decided = [((c, r), O.decide(self.stores[r], self.tab[r], self._id(c), has, wants, sub, now))
                   for c, r, has, wants, sub in requests]  # Decide + Assign, in queue order
        out = {}
        for (c, r), lease in decided:  # a client's last request of the round is its ticket's lease
            t = self.tab[r]
            safe = t["safe_capacity"]
            safe = t["capacity"] / float(self.stores[r].count()) if np.isnan(safe) else safe  # resource.go:91-95
            out[(c, r)] = (lease.has, lease.expiry_ns, int(t["refresh_interval_s"]), safe, float(t["capacity"]))
        return out


def _check(srv, tickets, expect, label):
    for (c, r), t in tickets.items():
        g, e, refresh, safe, cap = expect[(c, r)]
        lease = srv.lease(t)
        assert abs(lease.capacity - g) <= 1e-9 * max(abs(g), cap), (label, c, r, lease.capacity, g)
        assert lease.expiry_time == e // W.NS, (label, c, r)
        assert lease.refresh_interval == refresh
        assert (np.isnan(safe) and np.isnan(lease.safe_capacity)) or \
            abs(lease.safe_capacity - safe) <= 1e-9 * max(abs(safe), 1.0), (label, r, lease.safe_capacity, safe)


@pytest.mark.parametrize("seed", range(3))
def test_rounds_match_the_reference_server_model(seed):
    """Clients join, refresh, change wants, release and stop refreshing (their
    leases expire and Clean drops them) on FairShare / ProportionalShare / Static /
    NoAlgorithm / learning resources; resources outgrow their rows.  Every round's
    leases equal the reference server model's (each request's Decide + Assign in
    queue order)."""
    rng = np.random.default_rng(500 + seed)
    kinds = [W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.FAIR_SHARE, W.STATIC, W.NO_ALGORITHM, W.PROPORTIONAL_SHARE]
    resources = {f"r{k}": {"kind": kd, "capacity": float(rng.choice([10.0, 100.0, 1234.5])),
                           "lease_length_s": int(rng.choice([6, 20])), "refresh_interval_s": 2}
                 for k, kd in enumerate(kinds)}
    resources["r1"]["safe_capacity"] = 7.5
    resources["r5"]["learning_end_ns"] = NOW + 7 * W.NS  # learning for the first rounds
    srv = _server(resources, slots=2)
    model = ServerModel(resources)
    clients = [f"c{i}" for i in range(40)]
    now = NOW
    for rnd in range(12):
        now += 3 * W.NS
        reqs, tickets = [], {}
        for c in rng.choice(clients, 25, replace=False):
            r = f"r{rng.integers(len(kinds))}"
            if (c, r) in tickets:
                continue
            cap = resources[r]["capacity"]
            wants = float(rng.uniform(0, cap / 4)) if rng.random() > 0.1 else float(round(cap / 8))
            has = float(rng.uniform(0, cap / 8))
            reqs.append((c, r, has, wants, 1))
            tickets[(c, r)] = srv.get_capacity(c, r, has, wants)
        rels = [(c, f"r{rng.integers(len(kinds))}") for c in rng.choice(clients, 3, replace=False)]
        rels = [x for x in rels if x not in tickets]
        for c, r in rels:
            srv.release_capacity(c, r)
        srv.tick(now)
        _check(srv, tickets, model.round(now, reqs, rels), f"seed={seed} round={rnd}")
        for r in resources:
            st = srv.resource(r)
            assert st["clients"] == model.clients(r)
            assert st["count"] == model.stores[r].count()
    srv.close()


def test_expired_leases_are_cleaned_and_capacity_returns():
    """A client that stops refreshing loses its lease after lease_length
    (store.go:169-181): the remaining client then gets the whole capacity.
    Round 1: a sees the empty store (80); b is decided after a's Assign: the
    deserved share 50, capped by the unused capacity 100 - 80 = 20.  Round 2: a
    shares with b's stored lease (FairShare 50).  Round 3: b has expired and a gets
    its 80."""
    res = {"res": {"kind": W.FAIR_SHARE, "capacity": 100.0, "lease_length_s": 10, "refresh_interval_s": 5}}
    srv = _server(res)
    model = ServerModel(res)
    a = srv.get_capacity("a", "res", 0.0, 80.0)
    b = srv.get_capacity("b", "res", 0.0, 80.0)
    srv.tick(NOW)
    exp = model.round(NOW, [("a", "res", 0.0, 80.0, 1), ("b", "res", 0.0, 80.0, 1)], [])
    assert exp[("a", "res")][0] == 80.0 and exp[("b", "res")][0] == 20.0
    assert srv.lease(a).capacity == 80.0 and srv.lease(b).capacity == 20.0
    assert srv.resource("res")["sum_has"] == 100.0
    a = srv.get_capacity("a", "res", 80.0, 80.0)  # b does not refresh
    srv.tick(NOW + 5 * W.NS)
    assert model.round(NOW + 5 * W.NS, [("a", "res", 80.0, 80.0, 1)], [])[("a", "res")][0] == 50.0
    assert srv.lease(a).capacity == 50.0  # b still holds 20
    assert srv.resource("res")["clients"] == 2
    a = srv.get_capacity("a", "res", 50.0, 80.0)
    srv.tick(NOW + 11 * W.NS)  # b's lease (NOW + 10 s) has expired
    assert srv.resource("res")["clients"] == 1
    assert srv.lease(a).capacity == 80.0
    srv.close()


def test_release_capacity_frees_the_share():
    """ProportionalShare, capacity 90.  Round 1: a sees the empty store (60, what it
    wants), b the store after a's Assign (min(60, 90 - 60) = 30), c what is left
    (0).  Round 2: c releases; a and b each get the equal share, 45 (a first: 45;
    then b: unused 90 - 75 + 30 = 45).  Round 3: 45 each again, and the store's
    SumHas is the whole capacity."""
    res = {"res": {"kind": W.PROPORTIONAL_SHARE, "capacity": 90.0}}
    srv = _server(res)
    model = ServerModel(res)
    t = [srv.get_capacity(c, "res", 0.0, 60.0) for c in "abc"]
    srv.tick(NOW)
    exp = model.round(NOW, [(c, "res", 0.0, 60.0, 1) for c in "abc"], [])
    assert [exp[(c, "res")][0] for c in "abc"] == [60.0, 30.0, 0.0]
    assert [srv.lease(x).capacity for x in t] == [60.0, 30.0, 0.0]
    srv.release_capacity("c", "res")
    for k, (now, has) in enumerate([(NOW + W.NS, (60.0, 30.0)), (NOW + 2 * W.NS, (45.0, 45.0))]):
        reqs = [(c, "res", h, 60.0, 1) for c, h in zip("ab", has)]
        t = [srv.get_capacity(c, "res", h, 60.0) for c, h in zip("ab", has)]
        srv.tick(now)
        exp = model.round(now, reqs, [("c", "res")] if k == 0 else [])
        assert [exp[(c, "res")][0] for c in "ab"] == [45.0, 45.0]
        assert [srv.lease(x).capacity for x in t] == [45.0, 45.0]
    st = srv.resource("res")
    assert st["clients"] == 2 and st["count"] == 2 and st["sum_has"] == 90.0
    srv.close()


def test_round_grants_stay_within_capacity():
    """a round's requests are decided one after another, each seeing the
    Assigns before it (res.mu, resource.go:103-104; store.go:153-167), so the
    grants of a round never exceed what the reference would give.  FairShare,
    capacity 100: new clients that each want 100 get 100, 0, 0, 0 in the first
    round (simplecluster/fair: the later client gets nothing until the earlier one
    gives some back), not 400; the same holds for ProportionalShare.  Every lease
    equals the sequential oracle replay, and the store's SumHas <= capacity."""
    for kind in (W.FAIR_SHARE, W.PROPORTIONAL_SHARE):
        res = {"res": {"kind": kind, "capacity": 100.0, "lease_length_s": 60, "refresh_interval_s": 5}}
        srv = _server(res, slots=2)
        model = ServerModel(res)
        now = NOW
        for rnd in range(4):
            reqs = [(c, "res", 0.0 if rnd == 0 else 25.0, 100.0, 1) for c in "abcd"]
            t = {(c, r): srv.get_capacity(c, r, h, w) for c, r, h, w, _ in reqs}
            srv.tick(now)
            exp = model.round(now, reqs, [])
            _check(srv, t, exp, f"kind={kind} round={rnd}")
            got = [srv.lease(t[(c, "res")]).capacity for c in "abcd"]
            assert sum(got) <= 100.0 + 1e-9, (kind, rnd, got)
            if rnd == 0:
                assert got == [100.0, 0.0, 0.0, 0.0], (kind, got)
            assert srv.resource("res")["sum_has"] <= 100.0 + 1e-9
            now += W.NS
        srv.close()


def test_repeated_request_sees_its_own_earlier_assign():
    """Two requests of one client in one round: the second is decided after the
    first's Assign (the reference serves them one after another), and the ticket of
    each gets its own lease; the store keeps the last."""
    res = {"res": {"kind": W.FAIR_SHARE, "capacity": 100.0, "lease_length_s": 60}}
    srv = _server(res)
    model = ServerModel(res)
    reqs = [("a", "res", 0.0, 30.0, 1), ("b", "res", 0.0, 90.0, 1), ("a", "res", 30.0, 80.0, 1)]
    t = [srv.get_capacity(c, r, h, w) for c, r, h, w, _ in reqs]
    srv.tick(NOW)
    leases = [model.round(NOW, [q], [])[(q[0], q[1])][0] for q in reqs]  # the same Decides, one at a time
    got = [srv.lease(x).capacity for x in t]
    assert got == leases, (got, leases)
    st = srv.resource("res")
    assert st["clients"] == 2 and st["count"] == model.stores["res"].count()
    assert abs(st["sum_has"] - model.stores["res"].sum_has()) <= 1e-12 * 100
    srv.close()


def test_one_request_sees_the_store_before_its_own_assign():
    """the reference decides a request on the store as it is -- the
    client's own old row included, not its new wants (algorithm.go:217,245).
    Capacity 100; A holds 10 (wants 10), B holds 30 (wants 60); A asks for 60:
    SumWants is 70 <= 100, so A gets min(60, 100 - 40 + 10) = 60, not the 50 a
    store already holding A's new wants would give."""
    res = {"res": {"kind": W.PROPORTIONAL_SHARE, "capacity": 100.0, "lease_length_s": 60,
                   "learning_end_ns": NOW + W.NS}}
    srv = _server(res)
    model = ServerModel(res)
    reqs = [("a", "res", 10.0, 10.0, 1), ("b", "res", 30.0, 60.0, 1)]  # learning: Learn grants the reported has
    t = {(c, r): srv.get_capacity(c, r, h, w) for c, r, h, w, _ in reqs}
    srv.tick(NOW)
    _check(srv, t, model.round(NOW, reqs, []), "learning round")
    assert srv.lease(t[("a", "res")]).capacity == 10.0 and srv.lease(t[("b", "res")]).capacity == 30.0
    t = {("a", "res"): srv.get_capacity("a", "res", 10.0, 60.0)}
    srv.tick(NOW + 2 * W.NS)
    expect = model.round(NOW + 2 * W.NS, [("a", "res", 10.0, 60.0, 1)], [])
    assert expect[("a", "res")][0] == 60.0
    assert srv.lease(t[("a", "res")]).capacity == 60.0
    srv.close()


def test_release_capacity_kat():
    """server_test.go:404-433: after ReleaseCapacity the resource's SumHas is 0; an
    unknown resource in the same call is ignored."""
    case = next(c for c in KATS["server"] if c["name"] == "TestReleaseCapacity")
    rel = case["release"]
    cfg = _res_cfg(case, NOW - W.NS // 2)
    cfg["safe_capacity"] = case["safe_capacity"]
    srv = _server({"resource": cfg})
    t = srv.get_capacity("client", "resource", rel["request"]["has"], rel["request"]["wants"])
    srv.tick(NOW)
    assert srv.lease(t).capacity == rel["request"]["has"]  # learning mode (lease length 2 s)
    assert srv.lease(t).safe_capacity == case["safe_capacity"]
    for r in rel["release_resources"]:
        srv.release_capacity("client", r)
    srv.tick(NOW + W.NS)
    st = srv.resource("resource")
    assert st["sum_has"] == rel["post_sum_has"] and st["clients"] == 0
    srv.close()


def test_tickets_of_an_earlier_round_are_not_served():
    """dm_server_lease answers only the last round's tickets."""
    from doorman_amd.server import ServerError
    srv = _server({"res": {"kind": W.FAIR_SHARE, "capacity": 10.0}})
    t = srv.get_capacity("a", "res", 0.0, 4.0)
    srv.tick(NOW)
    assert srv.lease(t).capacity == 4.0
    srv.tick(NOW + W.NS)  # a round without requests
    with pytest.raises(ServerError):
        srv.lease(t)
    srv.close()


@pytest.mark.parametrize("seed", range(4))
def test_decide_matches_sequential_oracle_decides(seed):
    """dm_decide against the oracle's literal Resource.Decide replayed request by
    request on each resource's store (each Decide ends with its Assign): existing
    clients with changed wants / subclients, new clients on free rows, a client
    asking twice, clients whose lease expired (Clean drops them first), learning
    mode, heterogeneous subclients, every kind; parity-mode running sums.  The
    device store itself is not changed."""
    from doorman_amd.engine import Engine
    rng = np.random.default_rng(900 + seed)
    snap = W.random_snapshot(rng, 30, 60, hetero=seed % 2 == 1, edge=seed == 3)
    N = len(snap["wants"])
    free = rng.random(N) < 0.15  # released rows: slots for new clients
    for k, v in (("wants", 0.0), ("has", 0.0), ("subclients", 0), ("expiry_ns", W.RELEASED)):
        snap[k][free] = v
    W.add_store_sums(snap)
    so = snap["seg_off"]
    rows = np.flatnonzero(rng.random(N) < 0.4)
    rows = np.concatenate([rows, rng.choice(rows, max(1, len(rows) // 10))])  # some clients ask twice
    rng.shuffle(rows)
    n = len(rows)
    cap_row = np.repeat(snap["capacity"], np.diff(so))
    wants = np.where(rng.random(n) < 0.5, snap["wants"][rows], rng.uniform(0, 2, n) * cap_row[rows] / 10)
    sub = np.where(rng.random(n) < 0.8, np.maximum(snap["subclients"][rows], 1), rng.integers(1, 5, n))
    has = rng.uniform(0, 1, n) * cap_row[rows] / 10
    with Engine(0) as e:
        e.load(snap)
        gets, exp = e.decide(NOW, rows, has, wants, sub)
        after = e.read_store()
    for k in ("has", "wants", "subclients", "expiry_ns"):  # the store is not changed
        np.testing.assert_array_equal(after[k], snap[k])
    cfg = O.make_cfg(len(so) - 1)
    for f in O.CFG_DTYPE.names:
        cfg[f] = snap[f]
    stores = {}
    ref_g, ref_e = np.empty(n), np.empty(n, np.int64)
    for k, row in enumerate(rows):
        r = int(np.searchsorted(so, row, side="right")) - 1
        if r not in stores:
            st = O.Store(int(so[r + 1] - so[r]))
            for j in range(so[r], so[r + 1]):
                if snap["expiry_ns"][j] != W.RELEASED:
                    st.put(int(j - so[r]), int(snap["expiry_ns"][j]), snap["has"][j], snap["wants"][j],
                           int(snap["subclients"][j]))
            st.set_sums(int(snap["agg_count"][r]), snap["agg_sum_has"][r], snap["agg_sum_wants"][r])
            stores[r] = st
        lease = O.decide(stores[r], cfg[r], int(row - so[r]), has[k], wants[k], int(sub[k]), NOW)
        ref_g[k], ref_e[k] = lease.has, lease.expiry_ns
    np.testing.assert_array_equal(exp, ref_e)
    ok = float_close(gets, ref_g, cap_row[rows])
    assert ok.all(), (np.flatnonzero(~ok)[:8], gets[~ok][:4], ref_g[~ok][:4])


def _oracle_round(snap, rows, has, wants, sub, now, limit=None):
    """The oracle's literal Resource.Decide replayed request by request on each
    resource's store, each ending with its Assign (resource.go:100-113); the first
    `limit` requests only when given (a prefix of a round is decided exactly as in the
    whole round)."""
    so = snap["seg_off"]
    cfg = O.make_cfg(len(so) - 1)
    for f in O.CFG_DTYPE.names:
        cfg[f] = snap[f]
    n = len(rows) if limit is None else min(limit, len(rows))
    stores = {}
    ref_g, ref_e = np.empty(n), np.empty(n, np.int64)
    for k in range(n):
        row = rows[k]
        r = int(np.searchsorted(so, row, side="right")) - 1
        if r not in stores:
            st = O.Store(int(so[r + 1] - so[r]))
            for j in range(so[r], so[r + 1]):
                if snap["expiry_ns"][j] != W.RELEASED:
                    st.put(int(j - so[r]), int(snap["expiry_ns"][j]), snap["has"][j], snap["wants"][j],
                           int(snap["subclients"][j]))
            st.set_sums(int(snap["agg_count"][r]), snap["agg_sum_has"][r], snap["agg_sum_wants"][r])
            stores[r] = st
        lease = O.decide(stores[r], cfg[r], int(row - so[r]), has[k], wants[k], int(sub[k]), now)
        ref_g[k], ref_e[k] = lease.has, lease.expiry_ns
    return ref_g, ref_e


def _fast_round_snapshot(rng, sizes, kinds, s0):
    """Resources whose live rows all hold one subclients count (per resource), every
    row live: rounds of existing clients refreshing with that count take the fast path."""
    N = int(np.sum(sizes))
    R = len(sizes)
    cap = rng.choice([100.0, 1000.0, 12345.678], R)
    cap_row = np.repeat(cap, sizes)
    sub = np.repeat(np.asarray(s0), sizes).astype(np.int64)
    wants = rng.uniform(0.0, 3.0, N) * cap_row / np.repeat(np.maximum(sizes, 1), sizes) * sub
    tie = rng.random(N) < 0.1
    wants[tie] = np.round(wants[tie])
    has = rng.uniform(0.0, 1.2, N) * cap_row / np.repeat(np.maximum(sizes, 1), sizes)
    snap = W.make_snapshot(sizes, wants, has, sub, NOW + 600 * W.NS, np.asarray(kinds, np.int32), cap, 20, 5)
    return W.add_store_sums(snap)


def _decide_engine(fast=True):
    from doorman_amd.engine import Engine
    old = os.environ.get("DM_DECIDE_FAST")
    os.environ["DM_DECIDE_FAST"] = "1" if fast else "0"
    try:
        return Engine(0)
    finally:
        if old is None:
            os.environ.pop("DM_DECIDE_FAST")
        else:
            os.environ["DM_DECIDE_FAST"] = old


@pytest.mark.parametrize("seed", range(3))
def test_decide_fast_path_matches_sequential_oracle(seed):
    """dm_decide's fast path (dm_decide_fast.hip: resources with >= 64 requests whose
    requests keep every count) against the oracle's literal replay of the whole round,
    and against the one-workgroup replay (DM_DECIDE_FAST=0): FairShare and
    ProportionalShare resources of several sizes, rounds of one request per client
    (the grants' recurrence as a scan of max-plus maps) and of 1-3 requests per client
    (clients asking twice see their own earlier Assign), wants unchanged, new, tied,
    subclient counts 1 and 3, rounds longer than one event block (2048 requests);
    one resource gets a request with another count (the fast path declines it) and
    one holds released rows asked for again (declined too)."""
    rng = np.random.default_rng(31 + seed)
    sizes = np.array([3000, 700, 1500, 90, 40, 2600], dtype=np.int64)
    kinds = [W.FAIR_SHARE, W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.FAIR_SHARE, W.PROPORTIONAL_SHARE, W.FAIR_SHARE]
    s0 = [1, 3, 1, 3, 1, 1]
    snap = _fast_round_snapshot(rng, sizes, kinds, s0)
    so = snap["seg_off"]
    # resource 5: a tenth of its rows released (requests for them are new clients: declined)
    rel = so[5] + rng.choice(sizes[5], sizes[5] // 10, replace=False)
    snap["expiry_ns"][rel] = W.RELEASED
    snap["has"][rel] = 0.0
    snap["wants"][rel] = 0.0
    snap["subclients"][rel] = 0
    W.add_store_sums(snap)
    rows, wants, sub = [], [], []
    for r, n in enumerate(sizes):
        if r % 2 == 0:  # every client once (the grants' recurrence as a scan)
            rr = so[r] + rng.permutation(n)
            K = n
        else:  # some clients two or three times (the recurrence in order)
            K = int(n * rng.choice([1.0, 1.5, 2.5]))
            rr = so[r] + rng.integers(0, n, K)
        cw = snap["wants"][rr]
        fresh = rng.uniform(0.0, 3.0, K) * snap["capacity"][r] / n * s0[r]
        w = np.where(rng.random(K) < 0.4, cw, fresh)
        t = rng.random(K) < 0.1
        w[t] = np.round(w[t])
        rows.append(rr)
        wants.append(w)
        sub.append(np.full(K, s0[r], np.int64))
    rows, wants, sub = np.concatenate(rows), np.concatenate(wants), np.concatenate(sub)
    odd = np.flatnonzero((rows >= so[1]) & (rows < so[2]))[5]
    sub[odd] = 2  # resource 1: one request changes its count -> k_decide
    order = rng.permutation(len(rows))  # interleave the resources' requests
    rows, wants, sub = rows[order], wants[order], sub[order]
    has = rng.uniform(0, 1, len(rows))
    fast, slow = _decide_engine(True), _decide_engine(False)
    try:
        fast.load(snap)
        slow.load(snap)
        gets, exp = fast.decide(NOW, rows, has, wants, sub)
        again, _ = fast.decide(NOW, rows, has, wants, sub)
        sg, se = slow.decide(NOW, rows, has, wants, sub)
    finally:
        fast.close()
        slow.close()
    assert gets.tobytes() == again.tobytes(), "the fast path is deterministic"
    ref_g, ref_e = _oracle_round(snap, rows, has, wants, sub, NOW)
    cap_row = np.repeat(snap["capacity"], np.diff(so))
    np.testing.assert_array_equal(exp, ref_e)
    np.testing.assert_array_equal(se, ref_e)
    for got, label in ((gets, "fast"), (sg, "one-workgroup replay")):
        ok = float_close(got, ref_g, cap_row[rows])
        assert ok.all(), (label, np.flatnonzero(~ok)[:8], got[~ok][:4], ref_g[~ok][:4])
    e = np.max(np.abs(gets - ref_g) / np.maximum(np.abs(ref_g), cap_row[rows]))
    print(f"\nfast-path decide: {len(rows)} requests, max |got-ref|/max(|ref|, C) = {e:.3e} (bar 1e-9)")


def test_decide_100k_requests_on_a_100k_client_resource():
    """every client of a 100k-client FairShare resource refreshes in
    one round (new wants, same subclients), so the round is 100k requests on one
    resource -- 10^10 row visits for a request-by-request replay.  The fast path's
    device time (dm_kernel_times "decide") is reported and must stay under 10 ms; the
    first 3000 requests are checked against the oracle's literal replay (a prefix of a
    sequential round is decided exactly as in the whole round), the whole round's
    capacity bookkeeping by the grants' sum (asserted <= capacity, every grant >= 0),
    and a 9000-request round (several event blocks and scan chunks) request by request
    against the sequential replay."""
    rng = np.random.default_rng(5)
    n = 100_000
    snap = _fast_round_snapshot(rng, np.array([n], np.int64), [W.FAIR_SHARE], [1])
    rows = rng.permutation(n).astype(np.int64)
    wants = rng.uniform(0.0, 3.0, n) * snap["capacity"][0] / n
    sub = np.ones(n, np.int64)
    has = np.zeros(n)
    e = _decide_engine(True)
    try:
        e.load(snap)
        e.decide(NOW, rows[:100], has[:100], wants[:100], sub[:100])  # warm-up (allocations, code objects)
        e.set_profiling(True)
        e.reset_kernel_times()
        gets, exp = e.decide(NOW, rows, has, wants, sub)
        launches, ms = e.kernel_times()["decide"]
        e.set_profiling(False)
    finally:
        e.close()
    ref_g, ref_e = _oracle_round(snap, rows, has, wants, sub, NOW, limit=3000)
    cap = snap["capacity"][0]
    assert float_close(gets[:3000], ref_g, np.full(3000, cap)).all()
    np.testing.assert_array_equal(exp[:3000], ref_e)
    # the whole round's capacity bookkeeping: no grant negative, and the grants (every
    # client's lease after the round: each asked once) never exceed the capacity
    assert (gets >= 0).all()
    assert gets.sum() <= cap * (1 + 1e-12), (gets.sum(), cap)
    print(f"\n100k requests on a 100k-client resource: {ms:.2f} ms of device time (bar 10 ms); "
          f"sum of grants {gets.sum():.6f} of capacity {cap}")
    assert launches == 1 and ms < 10.0, ms
    # beyond the first 3000: a round of 9000 requests on the same resource (4 Assign-event
    # blocks of kFdBlock = 2048, 9 scan chunks of kFdChunk = 1024) decided by the fast path
    # and by the sequential replay (DM_DECIDE_FAST=0) must agree on every request
    k = 9000
    out = []
    for fast in (True, False):
        e = _decide_engine(fast)
        try:
            e.load(snap)
            out.append(e.decide(NOW, rows[:k], has[:k], wants[:k], sub[:k]))
        finally:
            e.close()
    (gf, ef), (gs, es) = out
    np.testing.assert_array_equal(ef, es)
    ok = float_close(gf, gs, np.full(k, cap))
    assert ok.all(), np.flatnonzero(~ok)[:10]
