"""Where a step's time goes: every kernel of a rocprofv3 --kernel-trace CSV (library
kernels, torch copies, runtime blits), in start order.

  python tools/step_trace.py gpurun_out/x/trace [--anchor k_block_dense] [--skip 30] [--show 3]

Steps are delimited by the anchor kernel's launches (one per step).  Per step: the
period (anchor start -> next anchor start), the GPU-idle time (no kernel running on
any queue) and, per kernel name, its median duration and the median gap before it
(from the previous kernel's end on the same queue).  --show prints the first steps
after --skip kernel by kernel.
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name):
    return name.split("(")[0].replace("void ", "").replace("dm::", "").split("<")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="k_block_dense")
    ap.add_argument("--skip", type=int, default=30)
    ap.add_argument("--show", type=int, default=2)
    args = ap.parse_args()
    path = args.csv
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = []
    for r in csv.DictReader(open(path)):
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), q))
    ks.sort()
    anchors = [i for i, k in enumerate(ks) if k[2] == args.anchor]
    if len(anchors) < args.skip + 3:
        raise SystemExit(f"{len(anchors)} {args.anchor} launches: too few")
    med = statistics.median
    periods, idle = [], []
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    last_end = {}
    for i, (s, e, n, q) in enumerate(ks):
        if q in last_end and anchors[args.skip] <= i:
            gap[n].append((s - last_end[q]) / 1e3)
        last_end[q] = e
    shown = 0
    for a, b in zip(anchors[args.skip:-1], anchors[args.skip + 1:]):
        t0, t1 = ks[a][0], ks[b][0]
        periods.append((t1 - t0) / 1e3)
        busy_until, idle_ns = t0, 0
        for s, e, n, q in ks[a:b]:
            dur[n].append((e - s) / 1e3)
            if s > busy_until:
                idle_ns += s - busy_until
            busy_until = max(busy_until, e)
        idle_ns += max(0, t1 - busy_until)
        idle.append(idle_ns / 1e3)
        if shown < args.show:
            shown += 1
            print(f"-- step at {t0}: period {(t1 - t0) / 1e3:.1f} us")
            for s, e, n, q in ks[a:b]:
                print(f"   q{q:>3s} {n:40s} start +{(s - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}")
    print(f"steps analysed: {len(periods)}; period median {med(periods):.1f} us (min {min(periods):.1f}), "
          f"GPU idle median {med(idle):.1f} us per step")
    print(f"{'kernel':40s} {'n/step':>6s} {'dur med':>8s} {'gap before (same queue) med':>28s}")
    nsteps = len(periods)
    for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        g = gap.get(n)
        print(f"{n:40s} {len(v) / nsteps:6.2f} {med(v):8.1f} {med(g) if g else float('nan'):28.1f}")


if __name__ == "__main__":
    main()
