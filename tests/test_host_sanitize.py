"""The host plugin surface (host/*.cpp: SparseMatrix, SoftwareSpMV, MatrixIO,
MatrixOps, Synthetic, csr2csc) built with AddressSanitizer and
UndefinedBehaviorSanitizer and driven over every reference fixture by
tools/host_check.cpp: golden.bin compare, preprocessing statistics,
transpose round trips, row permutation, .bin / Matrix Market I/O (including
malformed files), generators and partitions.  CPU only, no GPU calls."""
import os
import subprocess
import tempfile

import fixtures as fx
import hipspmv as hs


def test_host_surface_under_sanitizers():
    subprocess.run(["make", "-C", hs.PKG_DIR, "lib/host_check_san"], check=True, stdout=subprocess.DEVNULL)
    with tempfile.TemporaryDirectory() as tmp:
        out = subprocess.run([os.path.join(hs.LIB_DIR, "host_check_san"), fx.MATRICES, tmp, *fx.ALL_FIXTURES],
                             capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "host_check: 0 failures" in out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr
