"""Summarise a tools/gpu_profile.sh run into profiles/.

Reads rocprofv3 CSVs (kernel trace stats, FETCH_SIZE and WRITE_SIZE passes, and
the same counters on tools/ubench's k_flat8 kernel whose traffic is known) and
writes:
  profiles/pmc_<workload>.json   per kernel class: avg duration, raw counters,
                                 calibrated HBM bytes per launch (bench.py reads it)
  profiles/rocprof_<workload>.md the kernel-stats table and the derivation
Usage: python tools/pmc_summary.py gpurun_out/prof_<w> <w>
"""
import csv
import glob
import json
import os
import re
import sys

CLASS = [
    # template args <G, R[, BATCH]>: BATCH 2 is the HBM-streaming variant of the same bin
    (r"k_block_dense<128, 4>", "block128x4_dense"), (r"k_block_dense<128, 8>", "block128x8_dense"), (r"k_block_dense<64, 16>", "block128x8_dense"),
    (r"k_block_dense<256, 8>", "block256x8_dense"), (r"k_block_dense<512, 8>", "block2k4k_dense"),
    (r"k_block_dense<256, 16>", "block2k4k_dense"),
    (r"k_publish\b", "hier_publish"), (r"k_hier_tick\b", "hier_root"),
    (r"k_tick_done\b", "tick_done"), (r"k_count_undense\b", "count_undense"),
    (r"k_large_spec\b", "large_spec"), (r"k_large_redo(_team)?\b", "large_redo"),
    (r"k_block_rest<128, 4>", "block128x4_rest"), (r"k_block_rest<128, 8>", "block128x8_rest"), (r"k_block_rest<64, 16>", "block128x8_rest"),
    (r"k_block_rest<256, 8>", "block256x8_rest"), (r"k_block_rest<512, 8>", "block2k4k_rest"),
    (r"k_block_rest<256, 16>", "block2k4k_rest"),
    (r"k_large_t\b", "large_t"), (r"k_large_c_het\b", "large_c_het"), (r"k_large_e\b", "large_e"),
    (r"k_large_map_het\b", "large_map_het"),
    (r"k_block<128, 4(, \d)?>", "block128x4"), (r"k_block<128, 8(, \d)?>", "block128x8"), (r"k_block<64, 16>", "block128x8"), (r"k_block<256, 2(, \d)?>", "block256x2"), (r"k_block<256, 4(, \d)?>", "block256x4"),
    (r"k_block<256, 8(, \d)?>", "block256x8"), (r"k_block<512, 8(, \d)?>", "block2k4k"), (r"k_block<256, 16(, \d)?>", "block2k4k"), (r"k_block<512, 4(, \d)?>", "block512x4"), (r"k_block<1024, 4(, \d)?>", "block1024x4"),
    (r"k_wave<4(, \d)?>", "wave64x4"), (r"k_sub<16, 4>", "sub16x4"), (r"k_sub<32, 4>", "sub32x4"),
    (r"k_sub<8, 2>", "sub8x2"), (r"k_sub<16, 2>", "sub16x2"),
    (r"k_tile_small\b", "small_tiles"), (r"k_subs\b", "subs_merged"), (r"k_large_a\b", "large_a"), (r"k_large_b\b", "large_b"),
    (r"k_large_c\b", "large_c"), (r"k_large_map\b", "large_map"), (r"k_large_fin\b", "large_fin"),
    (r"k_general\b", "general"), (r"k_flat8\(", "ubench_flat8"), (r"k_flat8nt\(", "ubench_flat8nt"),
]


def cls(name):
    for pat, c in CLASS:
        if re.search(pat, name):
            return c
    return None


def find(d, suffix):
    hits = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    return hits[0] if hits else None


def counters(d):
    """mean counter value per dispatch, by kernel class"""
    f = find(d, "counter_collection.csv")
    if not f:
        return {}
    acc = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            c = cls(row.get("Kernel_Name", ""))
            if c is None:
                continue
            v = float(row.get("Counter_Value", 0) or 0)
            key = (c, row.get("Counter_Name"))
            s, n = acc.get(key, (0.0, 0))
            acc[key] = (s + v, n + 1)
    return {k: s / n for k, (s, n) in acc.items()}


def main(d, w):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats_f = find(os.path.join(d, "trace"), "kernel_stats.csv")
    stats = {}
    rows = []
    if stats_f:
        with open(stats_f) as fh:
            for row in csv.DictReader(fh):
                rows.append(row)
                c = cls(row["Name"])
                if c:  # several kernels of one class (e.g. k_large_redo's two builds): call-weighted
                    n, tot = int(row["Calls"]), float(row["TotalDurationNs"]) / 1e3
                    st = stats.setdefault(c, {"calls": 0, "total_us": 0.0})
                    st["calls"] += n
                    st["total_us"] += tot
                    st["avg_us"] = st["total_us"] / st["calls"]
    if not rows:
        sys.exit(f"no kernel stats under {d}/trace: not overwriting profiles/")
    fetch = counters(os.path.join(d, "fetch"))
    write = counters(os.path.join(d, "write"))
    cf = counters(os.path.join(d, "cal_fetch"))
    cw = counters(os.path.join(d, "cal_write"))
    # k_flat8 over 1e7 rows reads 32 B and writes 16 B per row
    known_r, known_w = 32 * 10_000_000, 16 * 10_000_000
    fr = cf.get(("ubench_flat8", "FETCH_SIZE"))
    wr = cw.get(("ubench_flat8", "WRITE_SIZE"))
    read_cal = known_r / (fr * 1024) if fr else 2.0  # guide: FETCH_SIZE reads 1/2 of wide streams
    write_cal = known_w / (wr * 1024) if wr else 1.0
    out = {"_calibration": {"read_factor": read_cal, "write_factor": write_cal,
                            "ubench_flat8_fetch_kb": fr, "ubench_flat8_write_kb": wr,
                            "note": "HBM bytes = FETCH_SIZE*1024*read_factor + WRITE_SIZE*1024*write_factor; factors "
                                    "from tools/ubench k_flat8 (8-byte lanes, 48 B/row known)"}}
    for (c, name), v in fetch.items():
        if name != "FETCH_SIZE" or c.startswith("ubench"):
            continue
        wv = write.get((c, "WRITE_SIZE"), 0.0)
        out[c] = {"fetch_kb": v, "write_kb": wv, "avg_us": stats.get(c, {}).get("avg_us"),
                  "hbm_bytes_per_launch": v * 1024 * read_cal + wv * 1024 * write_cal}
    # a split bin (k_block_dense + k_block_rest, one launch each per tick): the
    # class's bytes per tick include its rest kernel's
    for c in [k for k in out if k.endswith("_rest")]:
        base = c[: -len("_rest")]
        if base in out:
            out[base]["hbm_bytes_per_launch_dense_kernel"] = out[base]["hbm_bytes_per_launch"]
            out[base]["hbm_bytes_per_launch"] += out[c]["hbm_bytes_per_launch"]
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    with open(os.path.join(root, "profiles", f"pmc_{w}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    with open(os.path.join(root, "profiles", f"rocprof_{w}.md"), "w") as fh:
        fh.write(f"# rocprofv3 --kernel-trace --stats: bench.py --workload {w}\n\n")
        fh.write("| kernel | calls | avg (us) | min (us) | max (us) | share |\n|---|---|---|---|---|---|\n")
        for row in rows:
            fh.write(f"| `{row['Name'][:70]}` | {row['Calls']} | {float(row['AverageNs']) / 1e3:.2f} | "
                     f"{float(row['MinNs']) / 1e3:.2f} | {float(row['MaxNs']) / 1e3:.2f} | {row['Percentage']}% |\n")
        fh.write("\n## HBM traffic from PMC counters (separate --pmc passes)\n\n")
        fh.write(f"calibration (tools/ubench k_flat8, known 32 B read + 16 B written per row): "
                 f"read x{read_cal:.3f}, write x{write_cal:.3f}\n\n")
        fh.write("| kernel | FETCH_SIZE (KB) | WRITE_SIZE (KB) | HBM bytes / launch |\n|---|---|---|---|\n")
        for c, v in out.items():
            if c.startswith("_"):
                continue
            fh.write(f"| {c} | {v['fetch_kb']:.0f} | {v['write_kb']:.0f} | {v['hbm_bytes_per_launch']:.4g} |\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
