"""Per-dispatch durations of one hipspmv kernel from a rocprofv3 kernel-trace
CSV, in dispatch order (diagnostic for tools/warm_probe.py).

usage: warm_trace.py <kernel_trace.csv> [kernel-substring]
Prints one JSON line: the durations (us) in order and the gaps between
consecutive dispatches (us, end of one to start of the next)."""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_vcache<double, 3"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            if sub in name:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    dur = [round((e - b) / 1e3, 1) for b, e in rows]
    gap = [round((rows[i + 1][0] - rows[i][1]) / 1e3, 1) for i in range(len(rows) - 1)]
    print(json.dumps({"kernel": sub, "n": len(rows), "dur_us": dur, "gap_us": gap}))


if __name__ == "__main__":
    main()
