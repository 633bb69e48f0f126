#!/usr/bin/env python3
"""Per-counter summary of rocprofv3 --pmc counter CSVs for one kernel.

    python tools/pmc_summary.py OUT.csv KERNEL_SUBSTR pass1.csv [pass2.csv ...]

For every counter seen on dispatches whose Kernel_Name contains
KERNEL_SUBSTR: dispatches, the mean value per dispatch, and the mean per CU
(÷ 256; GRBM_* ÷ 8 XCDs: those count per XCD).  Derived rows where their
inputs are present: TCC hit rate, mean L1->L2 read latency (cycles) and the
requests in flight per CU by Little's law, LDS bank-conflict cycles per LDS
instruction, and HBM bytes per dispatch (FETCH_SIZE x 2 + WRITE_SIZE, KB ->
B, MI355X_MICROARCH.md §HBM).  The CSV is what profiles/ keeps and what the
plugin's counter-backed statistics read (option "pmc_csv")."""
import csv
import sys
from collections import defaultdict

CUS, XCDS = 256, 8


def summarize(substr, paths):
    vals = defaultdict(dict)  # counter -> {(path, dispatch): value}
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                if substr not in row.get("Kernel_Name", ""):
                    continue
                key = (path, row.get("Dispatch_Id"))
                vals[row["Counter_Name"]][key] = float(row["Counter_Value"])
    out = {}
    for name, d in sorted(vals.items()):
        mean = sum(d.values()) / len(d)
        per = XCDS if name.startswith("GRBM_") else CUS
        out[name] = {"dispatches": len(d), "per_dispatch": mean, "per_cu": mean / per}
    m = {k: v["per_dispatch"] for k, v in out.items()}
    derived = {}
    if "TCC_HIT" in m and "TCC_MISS" in m and m["TCC_HIT"] + m["TCC_MISS"] > 0:
        derived["tcc_hit_rate"] = m["TCC_HIT"] / (m["TCC_HIT"] + m["TCC_MISS"])
    if m.get("TCP_TCC_READ_REQ"):
        if "TCP_TCC_READ_REQ_LATENCY" in m:
            derived["l1_l2_read_latency_cycles"] = m["TCP_TCC_READ_REQ_LATENCY"] / m["TCP_TCC_READ_REQ"]
            cycles = m.get("GRBM_GUI_ACTIVE")
            if cycles:
                derived["l1_l2_requests_in_flight_per_cu"] = m["TCP_TCC_READ_REQ_LATENCY"] / (cycles / XCDS) / CUS
    if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
        derived["lds_conflict_cycles_per_lds_inst"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
    if "FETCH_SIZE" in m:
        derived["hbm_bytes_per_dispatch"] = m["FETCH_SIZE"] * 1024 * 2 + m.get("WRITE_SIZE", 0.0) * 1024
    return out, derived


def main(argv):
    if len(argv) < 4:
        sys.exit(__doc__)
    out_path, substr, paths = argv[1], argv[2], argv[3:]
    out, derived = summarize(substr, paths)
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["counter", "dispatches", "per_dispatch", "per_cu"])
        for name, v in out.items():
            w.writerow([name, v["dispatches"], f"{v['per_dispatch']:.6g}", f"{v['per_cu']:.6g}"])
        for name, v in derived.items():
            w.writerow([name, "", f"{v:.6g}", ""])
    for name, v in list(out.items()) + [(k, {"per_dispatch": v}) for k, v in derived.items()]:
        print(f"{name:40s} {v['per_dispatch']:.6g}")


if __name__ == "__main__":
    main(sys.argv)
