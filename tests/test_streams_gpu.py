"""The context's streams (round 5, dm_runtime.cpp take_aux / give_aux): a destroyed
context's whole stream set (its own stream, the four CU-masked auxiliary streams, the
copy stream) goes back to a per-device pool and the next context on the device gets
the earliest-created free set -- the hardware queues behind them are part of the tuning
 -- and the pool is destroyed at process exit."""
import os
import subprocess
import sys

import numpy as np
import pytest

from doorman_amd import workloads as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snap():
    rng = np.random.default_rng(5)
    sizes = rng.integers(1, 600, 300)
    N = int(sizes.sum())
    return W.make_snapshot(sizes, rng.uniform(0.5, 2.0, N), 0.0, 1, W.NOW_NS + 60 * W.NS, W.FAIR_SHARE, 100.0)


def test_a_destroyed_contexts_streams_go_to_the_next_context():
    import torch
    from doorman_amd.engine import Engine
    torch.cuda.set_device(0)
    snap = _snap()
    a = Engine(0)
    a.load(snap)
    a.apportion(W.NOW_NS, writeback=True)
    first = a.stream
    held = Engine(0)  # a second live context takes a set of its own
    assert held.stream != first
    a.close()
    b = Engine(0)  # the freed set, not a new one
    try:
        assert b.stream == first
        assert b.plan_info()["aux_own_queues"] == 1
        b.load(snap)
        b.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)
        b.apportion(W.NOW_NS + W.NS, writeback=True)
        gets, _ = b.leases()
        assert np.isfinite(gets).all()
    finally:
        b.close()
        held.close()


def test_the_process_exits_cleanly_with_pooled_streams():
    """Streams left in the pool are destroyed by the library's exit handler (a crash at
    exit under rocprofv3 otherwise); a process that created and closed contexts with
    deferred class work in flight exits with status 0."""
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, torch\n"
        "from doorman_amd import workloads as W\n"
        "from doorman_amd.engine import Engine\n"
        "torch.cuda.set_device(0)\n"
        "rng = np.random.default_rng(1); sizes = rng.integers(1, 3000, 400); N = int(sizes.sum())\n"
        "snap = W.make_snapshot(sizes, 1.0, 0.0, 1, W.NOW_NS + 60 * W.NS, W.FAIR_SHARE, 100.0)\n"
        "for k in range(3):\n"
        "    e = Engine(0); e.load(snap)\n"
        "    for t in range(4): e.apportion(W.NOW_NS + t * W.NS, writeback=True, asynchronous=True, defer_join=True)\n"
        "    e.close()\n"
        "keep = Engine(0); keep.load(snap); keep.apportion(W.NOW_NS, writeback=True, asynchronous=True, defer_join=True)\n"
        "print('done', flush=True)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "done" in r.stdout


def test_c2_tick_does_not_depend_on_streams_created_before_the_context():
    """a host that embeds the library (a cgo server) owns streams of its
    own.  configs[2]'s tick, in a process that first created 0, 1, 2 or 3 torch streams and
    used them, stays within 5 % of the clean process: each context times every assignment
    of its work classes to its four hardware queues on its first forked ticks and keeps
    the fastest (dm_plan_info queue_perm; the 24 assignments span 113-244 us per tick of
    calibration window, profiles/r06_queue_robustness.txt).  One process per case, one
    after another (tools/queue_probe.py)."""
    import json
    us = {}
    for k in (0, 1, 2, 3):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "queue_probe.py"), str(k), "torch", "600"],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (k, r.stderr[-2000:])
        line = json.loads(r.stdout.strip().splitlines()[-1])
        assert line["calibrated_perm"] is not None and line["calibrated_perm"] >= 0, line
        us[k] = line["us"]
    for k in (1, 2, 3):
        assert abs(us[k] / us[0] - 1.0) <= 0.05, us
