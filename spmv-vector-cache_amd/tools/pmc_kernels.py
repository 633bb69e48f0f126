#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one pass per CSV):
for every kernel whose name contains one of the given substrings, the mean
per dispatch of each counter, summed over the counter's instances.
usage: pmc_kernels.py 'substr1,substr2' csv...  (diagnostic)"""
import csv
import sys
from collections import defaultdict


def main():
    subs = sys.argv[1].split(",")
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    for f in sys.argv[2:]:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            hit = next((s for s in subs if s in name), None)
            if hit:
                per[hit][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in per.items():
        print(k)
        for c, d in sorted(cs.items()):
            vals = list(d.values())
            print(f"  {c:36s} {sum(vals) / len(vals):16.1f}  (per dispatch, {len(vals)} dispatches)")


if __name__ == "__main__":
    main()
