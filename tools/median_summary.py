#!/usr/bin/env python3
"""Medians of the repeated benchmark runs of tools/gpu_session.sh ``final_benches``
(BASELINE.md protocol: 3 runs of >= 200 timed steps).  Reads the last JSON line of every
``<dir>/fb_<name>_<run>.log`` and prints one JSON object: per benchmark the metric, unit,
median / min / max of ``value`` and ``ms_per_step``, and the runs' values.

Usage: python tools/median_summary.py [DIR]   (default gpurun_out)"""
import glob
import json
import os
import re
import statistics
import sys


def last_json(path):
    for line in reversed(open(path, errors="replace").read().splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    runs = {}
    for p in sorted(glob.glob(os.path.join(d, "fb_*_[0-9].log"))):
        m = re.match(r"fb_(.+)_(\d+)\.log$", os.path.basename(p))
        j = last_json(p)
        if m and j:
            runs.setdefault(m.group(1), []).append(j)
    out = {}
    for name, js in sorted(runs.items()):
        vals = [float(j["value"]) for j in js]
        ms = [float(j["ms_per_step"]) for j in js if j.get("ms_per_step") is not None]
        out[name] = {"metric": js[0]["metric"], "unit": js[0].get("unit"), "runs": len(js),
                     "steps": js[0].get("steps"), "value_median": statistics.median(vals),
                     "value_min": min(vals), "value_max": max(vals), "values": vals,
                     "ms_per_step_median": statistics.median(ms) if ms else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
