#!/usr/bin/env python
"""Roofline table from rocprofv3 passes over ``scripts/pmc_r3.py`` (one line per op).

usage: python scripts/pmc_summary.py --plan gpurun_out/pmc_r3_plan.json --trace DIR
                                     --pmc DIR [DIR ...] [--out profiles/r3_pmc_kernels.txt]

DIR = a rocprofv3 output directory (``*_kernel_trace.csv`` / ``*_counter_collection.csv``). Time
comes from the counter-free trace pass; counters are summed over the op's dispatches (between the
workload's int16 marker kernels) and divided by its call count.

Columns: time per call; achieved TF/s from the analytic FLOPs; MFMA FLOPs issued
(SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512) vs analytic; LDS bank-conflict cycles / LDS-active cycles;
HBM traffic (2 x FETCH_SIZE + WRITE_SIZE, KB counters; gfx950 FETCH_SIZE counts half the bytes
of wide reads) and its rate; arithmetic intensity and the
fraction of the roofline bound min(peak, AI x HBM) reached; MFMA-busy and LDS-busy cycles per
CU-cycle (GRBM_GUI_ACTIVE x 32 CUs per XCD; raw hardware ratios, not calibrated against a peak).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

PEAK_TF = 2500.0   # MI355X dense bf16 MFMA
HBM_TBS = 6.3      # measured streaming ceiling (MI355X_MICROARCH.md: 8 TB/s theoretical)


def _csv(d, suffix):
    f = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not f:
        raise SystemExit(f"no *{suffix} under {d}")
    return list(csv.DictReader(open(f[0])))


def _is_marker(name):
    return "short" in name and "add" in name.lower()


def _segments(dispatches):
    """dispatch list (id, name, payload) in launch order -> payload lists between marker pairs."""
    segs, cur, inside = [], None, False
    for _, name, payload in dispatches:
        if _is_marker(name):
            if inside:
                segs.append(cur)
            inside = not inside
            cur = []
        elif inside:
            cur.append((name, payload))
    return segs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plan", required=True)
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pmc", nargs="+", default=[])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    plan = json.load(open(a.plan))

    rows = _csv(a.trace, "kernel_trace.csv")
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    tsegs = _segments([(int(r["Dispatch_Id"]), r["Kernel_Name"],
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3) for r in rows])

    counters = [defaultdict(float) for _ in plan]
    for d in a.pmc:
        per = defaultdict(dict)
        names = {}
        for r in _csv(d, "counter_collection.csv"):
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[did] = r["Kernel_Name"]
        segs = _segments([(i, names[i], per[i]) for i in sorted(per)])
        for i, e in enumerate(plan):
            if i >= len(segs):
                break
            pat = re.compile(e["pattern"])
            for name, cvals in segs[i]:
                if pat.search(name):
                    for k, v in cvals.items():
                        counters[i][k] += v / e["calls"]

    lines = ["# r3 PMC roofline (1x MI355X, rocprofv3; per call = op total over its dispatches / calls)",
             f"# peaks: {PEAK_TF:.0f} TF/s dense bf16 MFMA, {HBM_TBS} TB/s HBM streaming",
             f"{'op':38s} {'us':>8s} {'TF/s':>7s} {'%pk':>5s} {'mfmaF/anl':>9s} {'ldsConf':>7s} "
             f"{'HBM MB':>8s} {'TB/s':>5s} {'AI':>6s} {'%roof':>6s} {'mfmaBusy':>8s} {'ldsBusy':>7s}  bound"]
    for i, e in enumerate(plan):
        pat = re.compile(e["pattern"])
        us = sum(t for n, t in tsegs[i] if pat.search(n)) / e["calls"] if i < len(tsegs) else float("nan")
        c = counters[i]
        tf = e["flops"] / (us * 1e-6) / 1e12 if us == us and us > 0 else float("nan")
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        mf = f"{mops * 512 / e['flops']:9.3f}" if mops else f"{'-':>9s}"
        lds = (c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]) if c.get("SQ_LDS_IDX_ACTIVE") else None
        ldss = f"{lds:7.3f}" if lds is not None else f"{'-':>7s}"
        # KB counters; gfx950's FETCH_SIZE tallies 128-B requests at 64 B, i.e. half the bytes of a
        # wide coalesced read (MI355X_MICROARCH.md §HBM): doubled here
        hbm = (2.0 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024.0
        if hbm <= 0:
            hbm = e["bytes"]
            src = "model"
        else:
            src = "pmc"
        tbs = hbm / (us * 1e-6) / 1e12 if us == us and us > 0 else float("nan")
        ai = e["flops"] / hbm
        roof = min(PEAK_TF, ai * HBM_TBS)
        bound = "MFMA" if ai * HBM_TBS >= PEAK_TF else "HBM"
        # busy fractions per CU-cycle: GRBM_GUI_ACTIVE counts GPU-active cycles per XCD (summed
        # over the 8), so x 32 CUs per XCD gives CU-cycles
        cu_cyc = c.get("GRBM_GUI_ACTIVE", 0) * 32
        mb = f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / cu_cyc:8.3f}" if cu_cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in c else f"{'-':>8s}"
        lb = f"{c['SQ_LDS_IDX_ACTIVE'] / cu_cyc:7.3f}" if cu_cyc and "SQ_LDS_IDX_ACTIVE" in c else f"{'-':>7s}"
        lines.append(f"{e['label']:38s} {us:8.1f} {tf:7.1f} {100 * tf / PEAK_TF:5.1f} {mf} {ldss} "
                     f"{hbm / 1e6:8.1f} {tbs:5.2f} {ai:6.0f} {100 * tf / roof:6.1f} {mb} {lb}  {bound} ({src} bytes)")
    # stall counters (a pass of their own): fractions of the op's wave-cycles
    stall = ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_LDS_DATA_FIFO_FULL", "SQ_LDS_CMD_FIFO_FULL"]
    if any(c.get("SQ_WAVE_CYCLES") and any(k in c for k in stall) for c in counters):
        lines.append("")
        lines.append(f"{'op':38s} " + " ".join(f"{k.replace('SQ_', '').lower():>18s}" for k in stall)
                     + "   (per wave-cycle)")
        for i, e in enumerate(plan):
            c = counters[i]
            if not c.get("SQ_WAVE_CYCLES"):
                continue
            lines.append(f"{e['label']:38s} " + " ".join(
                f"{c[k] / c['SQ_WAVE_CYCLES']:18.3f}" if k in c else f"{'-':>18s}" for k in stall))
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
