"""Dispatches of the last forward in a rocprofv3 kernel-trace CSV, in launch
order: index, kernel (short name), grid, duration in us; and per-kernel sums.
The forward is found as the last run of dispatches after the final gap of
more than --gap ms between kernels (the synchronize between forwards).

    python tools/trace_order.py TRACE.csv [--gap 1.0]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gap", type=float, default=1.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cut = 0
    for i in range(1, len(rows)):
        if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > a.gap * 1e6:
            cut = i
    tot = defaultdict(float)
    for i, r in enumerate(rows[cut:]):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        tot[name] += us
        print(f"{i:3d} {us:9.1f} {grid:>9s} {name}")
    print("--- per kernel")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{v:9.1f} {k}")
    print(f"{sum(tot.values()):9.1f} total")


if __name__ == "__main__":
    main()
