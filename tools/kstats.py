"""Top kernels of a rocprofv3 --stats kernel_stats.csv: share of kernel time, calls,
average us, name.   python tools/kstats.py <kernel_stats.csv> [--top 12]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    r = list(csv.DictReader(open(a.csv)))
    tot = sum(float(x["TotalDurationNs"]) for x in r)
    for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[: a.top]:
        print(f'{float(x["TotalDurationNs"]) / tot * 100:5.1f}% {x["Calls"]:>7} {float(x["AverageNs"]) / 1e3:8.1f} us  '
              f'{x["Name"][:110]}')
    print(f"total {tot / 1e6:.2f} ms over {sum(int(x['Calls']) for x in r)} launches")


if __name__ == "__main__":
    main()
