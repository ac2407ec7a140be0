"""Aggregate a rocprofv3 --pmc CSV (counter_collection.csv) per kernel name
substring: sum of each counter over the matching dispatches, plus derived
ratios when the counters are present.

usage: python tools/pmc_agg.py counter_collection.csv SUBSTRING [SUBSTRING ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    tot = {s: defaultdict(float) for s in subs}
    disp = {s: set() for s in subs}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            for s in subs:
                if s in name:
                    tot[s][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[s].add(row.get("Dispatch_Id"))
    for s in subs:
        t = tot[s]
        print(f"== {s}: {len(disp[s])} dispatches")
        for k in sorted(t):
            print(f"  {k:32s} {t[k]:.4g}")
        wc = t.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in t:
                    print(f"  {k}/WAVE_CYCLES = {t[k] / wc:.3f}")
        if t.get("SQ_BUSY_CYCLES") and t.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"  MFMA busy / SQ busy = {t['SQ_VALU_MFMA_BUSY_CYCLES'] / t['SQ_BUSY_CYCLES']:.3f}")
        if t.get("GRBM_GUI_ACTIVE") and t.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            print(f"  MFMA busy / (GUI_ACTIVE x 256 SIMD-groups) = "
                  f"{t['SQ_VALU_MFMA_BUSY_CYCLES'] / (t['GRBM_GUI_ACTIVE'] / 8 * 256):.3f}")


if __name__ == "__main__":
    main()
