"""Per-kernel instruction mix from tools/valu_profile.sh: VALU instructions per
wave and the VALU issue time they need on the whole chip (4 cycles per wave64
instruction per SIMD, 1024 SIMDs, 2.4 GHz) against the kernel's average duration.

  python tools/valu_summary.py gpurun_out/valu_c2
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import cls  # noqa: E402

SIMDS, CLK = 256 * 4, 2.4e9


def main(d):
    f = glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True)[0]
    acc = {}
    for row in csv.DictReader(open(f)):
        c = cls(row["Kernel_Name"]) or row["Kernel_Name"][:30]
        acc.setdefault(c, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    dur = {}
    t = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if t:
        for row in csv.DictReader(open(t[0])):
            c = cls(row["Name"]) or row["Name"][:30]
            dur[c] = float(row["AverageNs"]) / 1e3
    print(f"{'kernel':14s} {'waves':>8s} {'valu/wave':>9s} {'salu/wave':>9s} {'vmem/wave':>9s} {'lds/wave':>8s} "
          f"{'valu_us':>8s} {'avg_us':>8s}")
    for k, v in sorted(acc.items()):
        m = {n: sum(x) / len(x) for n, x in v.items()}
        w = m.get("SQ_WAVES", 0) or 1
        valu_us = m.get("SQ_INSTS_VALU", 0) * 4 / SIMDS / CLK * 1e6
        vm = m.get("SQ_INSTS_VMEM_RD", 0) + m.get("SQ_INSTS_VMEM_WR", 0)
        print(f"{k:14s} {w:8.0f} {m.get('SQ_INSTS_VALU', 0) / w:9.1f} {m.get('SQ_INSTS_SALU', 0) / w:9.1f} "
              f"{vm / w:9.1f} {m.get('SQ_INSTS_LDS', 0) / w:8.1f} {valu_us:8.2f} {dur.get(k, 0):8.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
