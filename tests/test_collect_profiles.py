"""tools/collect_profiles.py on a synthetic gpurun_out tree (CPU only): the
kernel_stats tables, bench lines and PMC passes land in profiles/rNN with a
README that lists them."""
import json
import os
import subprocess
import sys

import hipspmv as hs

TOOL = os.path.join(hs.PKG_DIR, "tools", "collect_profiles.py")


def test_collect_profiles(tmp_path):
    src, dst = tmp_path / "gpurun_out", tmp_path / "profiles" / "r02"
    (src / "prof" / "host" / "77").mkdir(parents=True)
    (src / "prof" / "host" / "77" / "run_kernel_stats.csv").write_text(
        '"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n'
        '"void hipspmv::k_vcache<double, 2>(int)",25,3600000,144000.0,99.0,140000,149000,1700.0\n'
        '"__amd_rocclr_copyBuffer",3,9000,3000.0,1.0,2600,4400,600.0\n')
    line = {"metric": "m", "value": 467.7, "config": {"workload": "C3", "kernel": "vcache_split"},
            "roofline": {"kernel_us": 143.5, "frac": 0.369}, "rocprof": {"avg_us": 144.0}}
    (src / "bench.log").write_text("[bench] rocprof leg ...\n" + json.dumps(line) + "\n")
    (src / "pmc" / "p1" / "h").mkdir(parents=True)
    (src / "pmc" / "p1" / "h" / "run_counter_collection.csv").write_text("Kernel_Name,Counter_Name\n")
    out = subprocess.run([sys.executable, TOOL, str(src), str(dst)], capture_output=True, text=True, check=True)
    assert "k_vcache<double, 2>" in out.stdout and "| 467.7 |" in out.stdout
    assert (dst / "kernel_stats_prof_host_77.csv").exists() and (dst / "pmc" / "pass1.csv").exists()
    assert (dst / "logs" / "bench.log").exists()
    assert json.loads((dst / "bench.jsonl").read_text())["value"] == 467.7
    readme = (dst / "README.md").read_text()
    assert "144.00" in readme and "0.369" in readme and "PMC passes: 1" in readme
