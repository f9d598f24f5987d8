#!/usr/bin/env python
"""Per-kernel PMC table from a rocprofv3 --pmc output directory: dispatches grouped by (kernel
name without arguments, grid size), every counter averaged per dispatch, plus derived ratios when
the counters are present: wait / issue-stall / active shares of SQ_WAVE_CYCLES, MFMA-busy per
busy cycle, LDS bank-conflict share of LDS-active cycles.

usage: python scripts/pmc_group.py DIR [--filter SUBSTR] [--min-us 0]"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)
    return re.sub(r"xddp::kernels::", "", n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    disp = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], f)
            d = disp.setdefault(k, {"name": short(r["Kernel_Name"]), "grid": int(r["Grid_Size"]),
                                    "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "c": {}})
            d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    groups = defaultdict(list)
    for d in disp.values():
        if a.filter in d["name"]:
            groups[(d["name"], d["grid"])].append(d)
    counters = sorted({c for d in disp.values() for c in d["c"]})
    for (name, grid), ds in sorted(groups.items(), key=lambda kv: -sum(d["ns"] for d in kv[1])):
        n = len(ds)
        avg = {c: sum(d["c"].get(c, 0.0) for d in ds) / n for c in counters}
        us = sum(d["ns"] for d in ds) / n / 1e3
        parts = [f"{name[:70]:70s} grid {grid:>9d} n {n:3d} {us:8.1f}us"]
        wc = avg.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for c, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "istall"), ("SQ_ACTIVE_INST_ANY", "act"),
                           ("SQ_WAIT_INST_LDS", "ldsst")):
                if c in avg:
                    parts.append(f"{lab} {avg[c] / wc * 100:5.1f}%")
        if avg.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            parts.append(f"mfma/busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / avg['SQ_BUSY_CYCLES']:.2f}")
        if avg.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in avg:
            parts.append(f"ldsconf {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE'] * 100:5.1f}%")
        parts.append(" ".join(f"{c}={avg[c]:.4g}" for c in counters if c in avg))
        print("  ".join(parts))


if __name__ == "__main__":
    main()
