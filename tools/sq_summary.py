"""Per-kernel SQ wave-state fractions from tools/sq_profile.sh output.

  python tools/sq_summary.py gpurun_out/sq_c2
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import cls  # noqa: E402


def main(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = {}
    for row in csv.DictReader(open(f)):
        c = cls(row["Kernel_Name"]) or row["Kernel_Name"][:30]
        acc.setdefault(c, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    print(f"{'kernel':14s} {'wave_cyc':>12s} {'wait_any':>8s} {'wait_ins':>8s} {'active':>8s} {'valu':>8s} {'lds':>8s} {'vmem':>8s}")
    for k, v in sorted(acc.items()):
        m = {n: sum(x) / len(x) for n, x in v.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        fr = lambda n: m.get(n, 0) / wc  # noqa: E731
        print(f"{k:14s} {wc:12.0f} {fr('SQ_WAIT_ANY'):8.2f} {fr('SQ_WAIT_INST_ANY'):8.2f} {fr('SQ_ACTIVE_INST_ANY'):8.2f} "
              f"{fr('SQ_ACTIVE_INST_VALU'):8.2f} {fr('SQ_ACTIVE_INST_LDS'):8.2f} {fr('SQ_ACTIVE_INST_VMEM'):8.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
