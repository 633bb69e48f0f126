#!/usr/bin/env python3
"""Cache-behaviour statistics of a HIPSpMV kernel from rocprofv3 PMC passes
(SURVEY.md §8(f) rank 3).

The FPGA NewCache backend reports its vector cache through statKeys
(software/HardwareSpMVNewCache.cpp:130-204): totalCycles, activeCycles,
readMisses, hazardStalls, ...  On MI355X the same questions are answered by
hardware counters; this tool reads the counter CSVs that
tools/pmc_session.sh collects (one counter group per rocprofv3 --pmc pass)
and prints, per kernel, the mean per dispatch under the reference's names
plus the GPU-native ones:

  totalCycles    GRBM_GUI_ACTIVE / XCDs   GPU clock cycles the kernel spanned
  activeCycles   SQ_BUSY_CYCLES / (XCDs x shader engines per XCD)
                                          cycles the sequencers were busy
  readMisses     TCC_MISS_sum             L2 misses (x panel + entry fetches)
  readHits       TCC_HIT_sum              L2 hits
  hazardStalls   SQ_LDS_BANK_CONFLICT     LDS bank-conflict cycles (the y/x LDS
                                          read-modify-write analogue of the
                                          FPGA's y hazard stalls)
  l2HitRate, waitFraction (SQ_WAIT_ANY / SQ_WAVE_CYCLES), hbmBytes
  (FETCH_SIZE x 2 + WRITE_SIZE: the gfx950 correction of MI355X_MICROARCH.md
  §HBM), durationUs (dispatch Start/End timestamps), clockGHz.

    python tools/cache_stats.py DIR_OR_CSV... [--kernel SUBSTR] [--xcds 8] [--se-per-xcd 4]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counters(paths, kernel_substr: str):
    """{counter: [per-dispatch value]}, and dispatch durations in ns, for the
    kernels whose name contains kernel_substr."""
    vals = defaultdict(dict)  # counter -> {dispatch: value}
    dur = {}
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_substr not in row.get("Kernel_Name", ""):
                    continue
                d = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[row["Counter_Name"]][d] = float(row["Counter_Value"])
                if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                    dur[d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return {k: list(v.values()) for k, v in vals.items()}, list(dur.values())


def mean(v):
    return sum(v) / len(v) if v else None


def cache_stats(paths, kernel_substr: str = "k_vcache", xcds: int = 8, se_per_xcd: int = 4) -> dict:
    c, dur = read_counters(paths, kernel_substr)
    m = {k: mean(v) for k, v in c.items()}
    out = {"kernel": kernel_substr, "dispatches": max((len(v) for v in c.values()), default=0)}
    if dur:
        out["durationUs"] = mean(dur) / 1e3
    if "GRBM_GUI_ACTIVE" in m:
        out["totalCycles"] = m["GRBM_GUI_ACTIVE"] / xcds
        if dur:
            out["clockGHz"] = out["totalCycles"] / mean(dur)
    if "SQ_BUSY_CYCLES" in m:
        out["activeCycles"] = m["SQ_BUSY_CYCLES"] / (xcds * se_per_xcd)
    hit, miss = m.get("TCC_HIT_sum", m.get("TCC_HIT")), m.get("TCC_MISS_sum", m.get("TCC_MISS"))
    if miss is not None:
        out["readMisses"] = miss
    if hit is not None:
        out["readHits"] = hit
    if hit is not None and miss is not None and hit + miss > 0:
        out["l2HitRate"] = hit / (hit + miss)
    if "SQ_LDS_BANK_CONFLICT" in m:
        out["hazardStalls"] = m["SQ_LDS_BANK_CONFLICT"]
    if "SQ_INSTS_LDS" in m:
        out["ldsInstructions"] = m["SQ_INSTS_LDS"]
    if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
        out["waitFraction"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in m:
        out["hbmBytes"] = m["FETCH_SIZE"] * 1024 * 2 + m.get("WRITE_SIZE", 0.0) * 1024
    return out


def expand(args):
    paths = []
    for a in args:
        if os.path.isdir(a):
            paths += sorted(glob.glob(os.path.join(a, "**", "*counter_collection*.csv"), recursive=True))
            paths += sorted(glob.glob(os.path.join(a, "pass*.csv")))
        else:
            paths.append(a)
    return sorted(set(paths))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("inputs", nargs="+")
    p.add_argument("--kernel", default="k_vcache")
    p.add_argument("--xcds", type=int, default=8)
    p.add_argument("--se-per-xcd", type=int, default=4)
    a = p.parse_args()
    print(json.dumps(cache_stats(expand(a.inputs), a.kernel, a.xcds, a.se_per_xcd), indent=1))


if __name__ == "__main__":
    main()
