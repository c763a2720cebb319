#!/usr/bin/env python3
"""Median duration per launch position within a step, from a rocprofv3 kernel trace
(csv).  Steps start at the kernel whose name contains --first.  Usage:
    python tools/trace_steps.py <run_kernel_trace.csv> [--first alias_sample] [--skip 20]"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="alias_sample")
    ap.add_argument("--skip", type=int, default=20)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]][a.skip:]
    per, spans, gaps = {}, [], []
    for s, e in zip(starts, starts[1:]):
        for k, i in enumerate(range(s, e)):
            r = rows[i]
            per.setdefault((k, name(r)), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            if i > s:
                gaps.append((int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3)
        spans.append((int(rows[e]["Start_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e3)
    tot = 0.0
    for (k, n), v in sorted(per.items()):
        m = statistics.median(v)
        tot += m
        print(f"{k:3d} {n:40s} median {m:8.2f} us  (n={len(v)})")
    print(f"sum of medians {tot:.2f} us; step span median {statistics.median(spans):.2f} us; "
          f"inter-launch gap median {statistics.median(gaps):.2f} us over {len(spans)} steps")


if __name__ == "__main__":
    main()
