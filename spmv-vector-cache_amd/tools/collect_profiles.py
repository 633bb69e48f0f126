#!/usr/bin/env python3
"""Copy the judged artefacts of a GPU session (gpurun_out/) into profiles/rNN/
and write its README table.

    python tools/collect_profiles.py gpurun_out profiles/r02

Collected: every rocprofv3 kernel_stats.csv (renamed after its run
directory), the bench JSON lines found in *.log files (one bench.jsonl), the
session, pytest, sweep and ablation logs, and the --pmc counter CSVs of
tools/pmc_session.sh (pass<i>.csv).  The README lists, per kernel_stats file,
the hipspmv kernels with calls and average / min / max duration, and per bench
line its value, kernel time, roofline fraction and the profiler's average
where the line carries one.  Existing files in the target are kept unless
--force."""
import argparse
import csv
import glob
import json
import os
import shutil


def kernel_rows(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            r = {k.strip().lower().replace("_", ""): v for k, v in r.items() if k}
            name = r.get("name") or r.get("kernelname") or ""
            if "hipspmv::" in name:
                rows.append((name, int(float(r["calls"])), float(r["averagens"]) / 1e3, float(r["minns"]) / 1e3,
                             float(r["maxns"]) / 1e3))
    return sorted(rows, key=lambda t: -t[1] * t[2])


def bench_lines(paths):
    out = []
    for p in paths:
        for line in open(p, errors="replace"):
            line = line.strip()
            if line.startswith("{") and '"metric"' in line:
                try:
                    out.append((os.path.basename(p), json.loads(line)))
                except json.JSONDecodeError:
                    pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    os.makedirs(os.path.join(a.dst, "logs"), exist_ok=True)

    def put(src, name):
        dst = os.path.join(a.dst, name)
        if not os.path.exists(dst) or a.force:
            shutil.copyfile(src, dst)
        return dst

    stats = []
    for p in sorted(glob.glob(os.path.join(a.src, "**", "*kernel_stats.csv"), recursive=True)):
        rel = os.path.relpath(os.path.dirname(p), a.src).replace(os.sep, "_").replace(".", "") or "root"
        stats.append((put(p, f"kernel_stats_{rel}.csv"), kernel_rows(p)))
    logs = sorted(glob.glob(os.path.join(a.src, "*.log")))
    for p in logs:
        put(p, os.path.join("logs", os.path.basename(p)))
    pmc = sorted(glob.glob(os.path.join(a.src, "pmc", "p*", "**", "*counter_collection.csv"), recursive=True))
    if pmc:
        os.makedirs(os.path.join(a.dst, "pmc"), exist_ok=True)
        for i, p in enumerate(pmc, 1):
            put(p, os.path.join("pmc", f"pass{i}.csv"))
    benches = bench_lines(logs)
    with open(os.path.join(a.dst, "bench.jsonl"), "w") as f:
        for _, b in benches:
            f.write(json.dumps(b) + "\n")

    md = [f"# {os.path.basename(os.path.normpath(a.dst))}: GPU session artefacts", "",
          f"Collected from `{a.src}` by `spmv-vector-cache_amd/tools/collect_profiles.py`.", ""]
    if stats:
        md += ["## rocprofv3 --kernel-trace --stats", "", "| file | kernel | calls | avg µs | min µs | max µs |",
               "|---|---|---|---|---|---|"]
        for path, rows in stats:
            for name, calls, avg, mn, mx in rows[:6]:
                short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                md.append(f"| `{os.path.basename(path)}` | `{short}` | {calls} | {avg:.2f} | {mn:.2f} | {mx:.2f} |")
        md.append("")
    if benches:
        md += ["## bench lines", "",
               "| log | workload | kernel | GFLOP/s | kernel µs | roofline frac | rocprof avg µs |",
               "|---|---|---|---|---|---|---|"]
        for log, b in benches:
            rf, rp = b.get("roofline", {}), b.get("rocprof") or {}
            md.append(f"| {log} | {b['config'].get('workload', '')[:40]} | {b['config'].get('kernel')} | "
                      f"{b['value']} | {rf.get('kernel_us')} | {rf.get('frac')} | {rp.get('avg_us', '')} |")
        md.append("")
    if pmc:
        md += [f"## PMC passes: {len(pmc)} counter CSVs under `pmc/`", ""]
    readme = os.path.join(a.dst, "README.md")
    if not os.path.exists(readme) or a.force:
        with open(readme, "w") as f:
            f.write("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
