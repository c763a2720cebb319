#!/usr/bin/env python3
"""Timeline of the last training steps from a rocprofv3 kernel trace.

Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [--last N] [--first-kernel tr_fwd]
Prints, for the last N steps (a step starts at each launch of --first-kernel), every
kernel's start offset from the step start, its duration, the idle gap before it, and the
step span, so launch / dependency gaps inside a hipGraph replay can be read directly.
"""
import argparse
import csv


def short(name):
    name = name.split("(")[0]
    for pre in ("void ", "euler_hip::"):
        name = name.replace(pre, "")
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--first-kernel", default="tr_fwd")
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if args.first_kernel in r[2]]
    if len(starts) < args.last + 1:
        print("not enough steps in the trace")
        return
    spans = []
    for si in range(len(starts) - 1):
        a, b = starts[si], starts[si + 1]
        spans.append((rows[b][0] - rows[a][0]) / 1000.0)
    print(f"{len(spans)} step periods; last 20 mean {sum(spans[-20:]) / len(spans[-20:]):.2f} us")
    for si in range(len(starts) - 1 - args.last, len(starts) - 1):
        a, b = starts[si], starts[si + 1]
        t0 = rows[a][0]
        print(f"--- step period {(rows[b][0] - t0) / 1000.0:.2f} us")
        prev_end = None
        busy_end = t0
        for s, e, n in rows[a:b]:
            gap = (s - busy_end) / 1000.0 if s > busy_end else 0.0
            print(f"  +{(s - t0) / 1000.0:7.2f}  dur {(e - s) / 1000.0:6.2f}  idle-before {gap:5.2f}  {n}")
            busy_end = max(busy_end, e)
            prev_end = e
        del prev_end


if __name__ == "__main__":
    main()
