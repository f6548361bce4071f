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
    """The reference server's per-resource stores, decided per round on one
    snapshot by the CPU oracle (test infrastructure)."""

    def __init__(self, resources):
        self.ids = list(resources)
        self.cfg = resources
        self.leases = {r: {} for r in self.ids}  # client -> [has, wants, sub, expiry]

    def round(self, now, requests, releases):
        for r in self.ids:  # Clean (store.go:169-181)
            for c in [c for c, l in self.leases[r].items() if now > l[3]]:
                del self.leases[r][c]
        for c, r in releases:  # ReleaseCapacity (store.go:142-151)
            self.leases[r].pop(c, None)
        for c, r, has, wants, sub in requests:
            learning = self.cfg[r].get("learning_end_ns", I64_MIN) > now
            lease = self.leases[r].setdefault(c, [0.0, 0.0, 0, now])
            lease[0] = has if learning else lease[0]
            lease[1], lease[2] = wants, sub
        sizes, rows = [], []
        for r in self.ids:
            sizes.append(len(self.leases[r]))
            rows += [(r, c, *l) for c, l in self.leases[r].items()]
        col = lambda k, dt: np.array([x[k] for x in rows], dt)  # noqa: E731
        cfg = lambda f, d: [self.cfg[r].get(f, d) for r in self.ids]  # noqa: E731
        snap = W.make_snapshot(sizes, col(3, np.float64), col(2, np.float64), col(4, np.int64), col(5, np.int64),
                               cfg("kind", 0), cfg("capacity", 0.0), cfg("lease_length_s", 300),
                               cfg("refresh_interval_s", 5), cfg("learning_end_ns", I64_MIN),
                               cfg("parent_expiry_ns", I64_MAX), cfg("safe_capacity", np.nan))
        ref = O.apportion(snap, now)
        where = {(x[0], x[1]): i for i, x in enumerate(rows)}
        out = {}
        for c, r, *_ in requests:
            i = where[(r, c)]
            lease = self.leases[r][c]
            lease[0], lease[3] = ref["gets"][i], ref["expiry_ns"][i]
            k = self.ids.index(r)
            out[(c, r)] = (ref["gets"][i], ref["expiry_ns"][i], self.cfg[r].get("refresh_interval_s", 5),
                           ref["res_safe_capacity"][k], self.cfg[r]["capacity"])
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
    leases equal the model's, decided by the oracle on the same snapshot."""
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
            assert st["clients"] == len(model.leases[r])
            assert st["count"] == sum(l[2] for l in model.leases[r].values())
    srv.close()


def test_expired_leases_are_cleaned_and_capacity_returns():
    """A client that stops refreshing loses its lease after lease_length
    (store.go:169-181): the remaining client then gets the whole capacity."""
    srv = _server({"res": {"kind": W.FAIR_SHARE, "capacity": 100.0, "lease_length_s": 10, "refresh_interval_s": 5}})
    a = srv.get_capacity("a", "res", 0.0, 80.0)
    b = srv.get_capacity("b", "res", 0.0, 80.0)
    srv.tick(NOW)
    assert srv.lease(a).capacity == 50.0 and srv.lease(b).capacity == 50.0
    a = srv.get_capacity("a", "res", 50.0, 80.0)  # b does not refresh
    srv.tick(NOW + 5 * W.NS)
    assert srv.lease(a).capacity == 50.0  # b still holds 50
    assert srv.resource("res")["clients"] == 2
    a = srv.get_capacity("a", "res", 50.0, 80.0)
    srv.tick(NOW + 11 * W.NS)  # b's lease (NOW + 10 s) has expired
    assert srv.resource("res")["clients"] == 1
    assert srv.lease(a).capacity == 80.0
    srv.close()


def test_release_capacity_frees_the_share():
    srv = _server({"res": {"kind": W.PROPORTIONAL_SHARE, "capacity": 90.0}})
    t = [srv.get_capacity(c, "res", 0.0, 60.0) for c in "abc"]
    srv.tick(NOW)
    assert [srv.lease(x).capacity for x in t] == [30.0, 30.0, 30.0]
    srv.release_capacity("c", "res")
    t = [srv.get_capacity(c, "res", 30.0, 60.0) for c in "ab"]
    srv.tick(NOW + W.NS)
    assert [srv.lease(x).capacity for x in t] == [45.0, 45.0]
    st = srv.resource("res")
    assert st["clients"] == 2 and st["count"] == 2 and st["sum_has"] == 90.0
    srv.close()
