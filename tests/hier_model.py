"""Host-side reference model of one hierarchy exchange (test infrastructure):
builds the root server's store exactly as GetServerCapacity would see the
intermediate servers' requests (server.go:234-255 -> :850-879) and evaluates it
with the oracle."""
import numpy as np

from doorman_amd import workloads as W
from oracle import oracle as O


def leaf_totals(snap, now):
    """What each intermediate publishes per resource: store SumWants and Count after Clean."""
    out = O.apportion(snap, now)
    return out["res_sum_wants"], out["res_count"]


def root_from_totals(totals, capacity, kind, lease_length_s, prev_has, now):
    """totals: list over servers g of (sum_wants[R], count[R]).  Rows of servers that do
    not request (SumWants <= 0 or Count < 1) are released."""
    G = len(totals)
    R = len(totals[0][0])
    wants = np.zeros(R * G)
    sub = np.zeros(R * G, np.int64)
    exp = np.full(R * G, W.RELEASED, np.int64)
    has = np.zeros(R * G)
    for g, (sw, cnt) in enumerate(totals):
        for r in range(R):
            i = r * G + g
            if sw[r] > 0 and cnt[r] >= 1:
                wants[i], sub[i], exp[i], has[i] = sw[r], cnt[r], now, prev_has[i]
    snap = W.make_snapshot(np.full(R, G), wants, has, sub, exp, kind, capacity, lease_length_s, 5)
    return snap


def grants(root_snap, root_out, G, g):
    """server.go:284-296: capacity = gets, parent expiry = Unix seconds of the lease expiry."""
    R = len(root_snap["seg_off"]) - 1
    idx = np.arange(R) * G + g
    e = root_out["expiry_ns"][idx]
    live = e != W.RELEASED
    cap = root_out["gets"][idx]
    parent = np.where(live, (e // W.NS) * W.NS, W.INT64_MAX)
    return cap, parent, live
