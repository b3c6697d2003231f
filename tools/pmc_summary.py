"""Condense rocprofv3 ``--pmc`` counter CSVs into one per-kernel table.

usage: python tools/pmc_summary.py OUT.txt DIR [DIR ...]   (each DIR holds run_counter_collection.csv)
Per kernel (name cut at the first '(' / 90 chars): dispatch count and the sum of every counter;
derived ratios when their counters are present (MFMA busy share of GRBM_GUI_ACTIVE x CUs, LDS bank
conflict rate, L2 hit rate).
"""
import collections
import csv
import os
import sys


def short(name):
    n = name[5:] if name.startswith("void ") else name
    n = n.replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n[:90]


def main(out, dirs):
    agg = collections.OrderedDict()
    for d in dirs:
        seen = set()
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            k = short(r["Kernel_Name"])
            e = agg.setdefault(k, {"dispatches": 0})
            if (d, r["Dispatch_Id"]) not in seen:
                seen.add((d, r["Dispatch_Id"]))
                if d == dirs[0]:
                    e["dispatches"] += 1
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    lines = []
    for k, e in agg.items():
        parts = [f"{c}={v:.4g}" for c, v in e.items()]
        if e.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in e:
            parts.append(f"mfma_busy/(gui_active*256CU)={e['SQ_VALU_MFMA_BUSY_CYCLES'] / (e['GRBM_GUI_ACTIVE'] * 256):.3f}")
        if e.get("SQ_LDS_IDX_ACTIVE"):
            parts.append(f"lds_conflict_rate={e.get('SQ_LDS_BANK_CONFLICT', 0) / e['SQ_LDS_IDX_ACTIVE']:.3f}")
        if e.get("TCC_HIT_sum") is not None and e.get("TCC_MISS_sum") is not None:
            tot = e["TCC_HIT_sum"] + e["TCC_MISS_sum"]
            if tot:
                parts.append(f"l2_hit={e['TCC_HIT_sum'] / tot:.3f}")
        lines.append(f"{k}\n    " + "  ".join(parts))
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(open(out).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
