"""Per-tick timeline of a multi-stream tick from a rocprofv3 --kernel-trace CSV.

  python tools/timeline.py gpurun_out/tl/run_kernel_trace.csv [--skip 20]

Kernel k's i-th launch belongs to tick i (every kernel of the plan launches once per
tick).  Per work class (the queue the kernels ran on): busy time (sum of kernel
durations), span (first start -> last end) and the gaps between dependent launches;
per tick: the period (tick i+1's first start - tick i's first start) and which class
ended last.
"""
import argparse
import collections
import csv
import glob
import os
import statistics


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("dm::", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=int, default=20, help="ticks to skip (warm-up)")
    args = ap.parse_args()
    path = args.csv
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        name = short(r["Kernel_Name"])
        if not name.startswith("k_"):
            continue
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q))
    ks.sort()
    counts = collections.Counter(n for _, _, n, _ in ks)  # kernels of every tick only (not the
    top = max(counts.values())                            # occasional split-form retries)
    ks = [k for k in ks if counts[k[2]] >= top // 2]
    occ = collections.Counter()
    ticks = collections.defaultdict(list)
    for s, e, n, q in ks:
        ticks[occ[n]].append((s, e, n, q))
        occ[n] += 1
    nt = min(occ.values())
    idx = [i for i in range(args.skip, nt - 1)]
    per_class_busy = collections.defaultdict(list)
    per_class_span = collections.defaultdict(list)
    per_class_gap = collections.defaultdict(list)
    per_kernel = collections.defaultdict(list)
    last_class = collections.Counter()
    periods, spans = [], []
    for i in idx:
        t = ticks[i]
        t0 = min(s for s, _, _, _ in t)
        t1 = max(e for _, e, _, _ in t)
        periods.append((min(s for s, _, _, _ in ticks[i + 1]) - t0) / 1e3)
        spans.append((t1 - t0) / 1e3)
        byq = collections.defaultdict(list)
        for s, e, n, q in t:
            byq[q].append((s, e, n))
            per_kernel[n].append((e - s) / 1e3)
        ends = {}
        for q, L in byq.items():
            L.sort()
            label = "+".join(sorted({n for _, _, n in L}))[:60]
            per_class_busy[label].append(sum(e - s for s, e, _ in L) / 1e3)
            per_class_span[label].append((L[-1][1] - L[0][0]) / 1e3)
            per_class_gap[label].append(sum(max(0, L[j + 1][0] - L[j][1]) for j in range(len(L) - 1)) / 1e3)
            ends[label] = L[-1][1]
        last_class[max(ends, key=ends.get)] += 1
    med = statistics.median
    print(f"ticks analysed: {len(idx)}; period med {med(periods):.1f} us, span (first start -> last end) med {med(spans):.1f} us")
    print(f"{'class (queue)':62s} {'busy':>7s} {'span':>7s} {'gaps':>7s} last")
    for k in sorted(per_class_span, key=lambda k: -med(per_class_span[k])):
        print(f"{k:62s} {med(per_class_busy[k]):7.1f} {med(per_class_span[k]):7.1f} {med(per_class_gap[k]):7.1f} {last_class[k]}")
    print("per kernel (median us):")
    for n, v in sorted(per_kernel.items(), key=lambda kv: -med(kv[1])):
        print(f"  {n:40s} {med(v):7.1f}")


if __name__ == "__main__":
    main()
