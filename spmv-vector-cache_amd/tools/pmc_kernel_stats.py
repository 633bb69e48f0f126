#!/usr/bin/env python3
"""Per-kernel duration statistics from the Start/End dispatch timestamps that
rocprofv3 writes into its --pmc counter CSVs, in the column layout of
rocprofv3's --stats kernel_stats.csv (Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs, StdDev).  Each dispatch is counted once
per pass (a dispatch carries one row per counter).  Counter collection
serializes dispatches, so these durations can run slightly long compared with
a --kernel-trace run.

    python tools/pmc_kernel_stats.py OUT.csv pass1.csv [pass2.csv ...]
"""
import csv
import math
import sys
from collections import defaultdict


def main(argv):
    out, paths = argv[1], argv[2:]
    durs = defaultdict(list)
    for path in paths:
        seen = set()
        with open(path) as f:
            for row in csv.DictReader(f):
                key = row["Dispatch_Id"]
                if key in seen:
                    continue
                seen.add(key)
                durs[row["Kernel_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    total_all = sum(sum(v) for v in durs.values())
    rows = []
    for name, v in durs.items():
        n, tot = len(v), sum(v)
        avg = tot / n
        sd = math.sqrt(sum((d - avg) ** 2 for d in v) / n)
        rows.append([name, n, tot, avg, 100.0 * tot / total_all, min(v), max(v), sd])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in rows:
            w.writerow(r)
    for r in rows:
        print(f"{r[1]:5d} calls  avg {r[3] / 1e3:9.2f} us  min {r[5] / 1e3:9.2f}  max {r[6] / 1e3:9.2f}  {r[0][:90]}")


if __name__ == "__main__":
    main(sys.argv)
