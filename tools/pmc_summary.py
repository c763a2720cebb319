#!/usr/bin/env python3
"""Summarise the per-dispatch csv files written by tools/pmc_passes.sh into one per-kernel
table: dispatches, mean duration, HBM-side bytes (FETCH_SIZE + WRITE_SIZE, KiB in the
counters), achieved TB/s, MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE
x 1024 SIMDs, the rocprofv3 ``MfmaUtil`` derivation) and LDS bank-conflict cycles per LDS
instruction.  Durations come from the FETCH_SIZE pass (one counter group, small overhead).

Usage: python tools/pmc_summary.py gpurun_out/pmc_<name> [--top N] [--skip-first K]
"""
from __future__ import annotations

import argparse
import csv
import os
import re
from collections import defaultdict

SIMDS = 256 * 4


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:70]


def load(path):
    rows = defaultdict(lambda: defaultdict(float))     # dispatch -> counter -> value
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = (short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return rows, meta


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--top", type=int, default=15)
    args = p.parse_args()
    passes = {}
    for sub in sorted(os.listdir(args.dir)):
        f = os.path.join(args.dir, sub, "run_counter_collection.csv")
        if os.path.exists(f):
            passes[sub] = load(f)
    agg = defaultdict(lambda: defaultdict(float))
    for sub, (rows, meta) in passes.items():
        for d, cs in rows.items():
            k, dur = meta[d]
            a = agg[k]
            if sub == "FETCH_SIZE":
                a["n"] += 1
                a["t"] += dur
            for c, v in cs.items():
                a[c] += v
    order = sorted(agg.items(), key=lambda kv: -kv[1]["t"])[: args.top]
    total_t = sum(a["t"] for a in agg.values())
    print(f"| kernel | calls | mean us | % time | MB read | MB written | TB/s | MFMA util % | LDS confl/instr |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, a in order:
        n = max(a["n"], 1)
        rd = a["FETCH_SIZE"] * 1024 / n
        wr = a["WRITE_SIZE"] * 1024 / n
        t = a["t"] / n
        bw = (rd + wr) / t / 1e12 if t > 0 else 0.0
        mf = 100 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] * SIMDS) if a["GRBM_GUI_ACTIVE"] else 0.0
        lc = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_INSTS_LDS"] if a["SQ_INSTS_LDS"] else 0.0
        print(f"| {k} | {int(a['n'])} | {t * 1e6:.1f} | {100 * a['t'] / total_t:.1f} | {rd / 1e6:.1f} | {wr / 1e6:.1f} "
              f"| {bw:.2f} | {mf:.1f} | {lc:.2f} |")


if __name__ == "__main__":
    main()
