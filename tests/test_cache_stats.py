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


R04 = os.path.join(os.path.dirname(hs.PKG_DIR), "profiles", "r04", "s1")


def _pmc_mean(path, kernel_sub, counter):
    import csv
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_sub in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals[row["Dispatch_Id"]] = float(row["Counter_Value"])
    return sum(vals.values()) / len(vals), len(vals)


def test_pmc_counter_reads_round4_csv():
    # hipspmv_pmc_counter (libhipspmv, no device) on the committed round-4 pass of the
    # product kernel: the mean per dispatch of each counter equals a plain CSV read
    path = os.path.join(R04, "pmc_c3_split_pass3.csv")
    for counter in ("TCC_MISS", "TCC_HIT", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"):
        want, n = _pmc_mean(path, "k_vcache<double, 3,", counter)
        got, gn = hs.pmc_counter(path, counter, "k_vcache<double, 3,")
        assert gn == n == 10 and got == pytest.approx(want, rel=1e-12), counter
    # no kernel filter: the hipspmv kernel with the most dispatches; the summary CSV form
    assert hs.pmc_counter(path, "TCC_MISS")[0] == pytest.approx(_pmc_mean(path, "k_vcache", "TCC_MISS")[0])
    summ = os.path.join(R04, "pmc_c3_split_summary.csv")
    assert hs.pmc_counter(summ, "TCC_MISS")[0] == pytest.approx(_pmc_mean(path, "k_vcache", "TCC_MISS")[0],
                                                                rel=1e-5)
    with pytest.raises(hs.HipSpMVError):
        hs.pmc_counter(path, "NO_SUCH_COUNTER")


def test_spmvbench_csv_row_carries_pmc_counters():
    # spmvbench --pmc: the counters reach the plugin's CSV row (readMisses <- TCC_MISS,
    # hazardStalls <- SQ_LDS_BANK_CONFLICT; the layout values under *Model), as the
    # reference reads its counters from the accelerator (HardwareSpMVNewCache.cpp:161-173).
    # Without a GPU the backend's run fails, and the row still carries the CSV's counters.
    import subprocess
    if hs.device_count() > 0:
        pytest.skip("with a device the row reports the counters of the kernel that ran (a -m gpu concern)")
    path = os.path.join(R04, "pmc_c3_split_pass3.csv")
    repo = os.path.dirname(hs.PKG_DIR)
    out = subprocess.run([os.path.join(hs.LIB_DIR, "spmvbench"), "--dir", os.path.join(repo, "tests", "golden",
                          "matrices"), "--confs", "hip", "--cms", "0", "--pmc", path, "circuit204"],
                         capture_output=True, text=True, timeout=120).stdout.splitlines()
    head = next(l for l in out if l.startswith("nnz,") or "readMisses" in l)
    keys = head.rstrip(",").split(",")
    row = [l for l in out if l.rstrip(",").endswith("circuit204")][-1].rstrip(",").split(",")
    rec = dict(zip(keys, row))
    assert "readMissesModel" in rec and "hazardStallsModel" in rec
    assert int(rec["readMisses"]) == round(_pmc_mean(path, "k_vcache", "TCC_MISS")[0])
    assert int(rec["hazardStalls"]) == round(_pmc_mean(path, "k_vcache", "SQ_LDS_BANK_CONFLICT")[0])
