"""CPU replay of k_sell (spmv-vector-cache_amd/tools/sell_sim.cpp) on the
product SELL layout (csrc/plan.cpp build_sell): every load index the kernel
forms in bounds, every row written exactly once, ORDERED bit-exact against
the CSR reference, FAST within the bound, u64 exact -- on stripe, R-MAT (hub
rows), ragged, multi-window, empty, single-row and single-column matrices.
The replay runs plain and under ASan/UBSan.  No GPU."""
import os
import subprocess

import hipspmv as hs


def _run(target, *args):
    subprocess.run(["make", "-C", hs.PKG_DIR, f"lib/{target}"], check=True, stdout=subprocess.DEVNULL)
    out = subprocess.run([os.path.join(hs.LIB_DIR, target), *args], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if "beta=" in l]
    assert lines and all(": ok" in l for l in lines), out.stdout
    assert "VIOLATION" not in out.stderr and "runtime error" not in out.stderr
    assert "ThreadSanitizer" not in out.stderr
    return lines


def test_sell_replay():
    lines = _run("sell_sim")
    assert len(lines) == 8 * 2 * 3
    assert any(l.startswith("split hubs") for l in lines)  # rows in several FAST pieces
    assert any("hubs=0" not in l for l in lines)  # the hub path is exercised


def test_sell_replay_under_sanitizers():
    _run("sell_sim_san", "small")


def test_sell_layout_build_threads_race_free():
    # build_sell fills its windows from several threads (csrc/plan.cpp)
    lines = _run("sell_sim_tsan", "small")
    assert lines
