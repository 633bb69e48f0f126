"""tools/cache_stats.py (the NewCache statKeys analogue from rocprofv3 PMC
passes) on the committed round-1 counter CSVs of the product kernel."""
import os
import sys

import pytest

import hipspmv as hs

sys.path.insert(0, os.path.join(hs.PKG_DIR, "tools"))
import cache_stats  # noqa: E402

R01 = os.path.join(os.path.dirname(hs.PKG_DIR), "profiles", "r01", "pmc_vcache_split")


def test_cache_stats_round1_vcache_split():
    st = cache_stats.cache_stats(cache_stats.expand([R01]), "k_vcache")
    assert st["dispatches"] == 13
    assert st["l2HitRate"] == pytest.approx(0.695, abs=0.002)
    assert st["readMisses"] == pytest.approx(4.14e6, rel=0.01)
    assert st["hbmBytes"] == pytest.approx(512.6e6, rel=0.01)  # ~1.2x the 423.6 MB algorithmic bytes
    assert 2.2 < st["clockGHz"] < 2.5
    assert 0 < st["activeCycles"] <= st["totalCycles"]
    assert 0.4 < st["waitFraction"] < 0.6


def test_cache_stats_other_kernel_empty():
    st = cache_stats.cache_stats(cache_stats.expand([R01]), "k_csr_lane")
    assert st["dispatches"] == 0 and "l2HitRate" not in st


def test_kernel_stats_from_pmc_matches_committed(tmp_path):
    # profiles/r01/kernel_stats_from_pmc.csv is reproducible from the committed
    # PMC passes, and its product-kernel average agrees with the bench's
    # HIP-event time for the same kernel and workload (143.5 us) within 2 %
    import csv
    import glob
    import os
    import subprocess
    import sys
    import hipspmv as hs
    prof = os.path.join(hs.REPO_DIR, "profiles", "r01")
    out = tmp_path / "stats.csv"
    subprocess.run([sys.executable, os.path.join(hs.PKG_DIR, "tools", "pmc_kernel_stats.py"), str(out),
                    *sorted(glob.glob(os.path.join(prof, "pmc_vcache_split", "pass*.csv")))],
                   check=True, capture_output=True)
    assert out.read_text() == open(os.path.join(prof, "kernel_stats_from_pmc.csv")).read()
    rows = {r["Name"]: r for r in csv.DictReader(open(out))}
    k = next(r for n, r in rows.items() if "k_vcache<double, 2," in n)
    assert abs(float(k["AverageNs"]) / 1e3 - 143.5) / 143.5 < 0.02
