"""INTEGRATION.md section B, built and run: the reference's own plugin classes
drive the HIP backend.

oracle/_ref/refbridge links the reference's software/SpMV.cpp,
HardwareSpMV.cpp, SparseMatrix.cpp and malloc_aligned.c -- compiled unmodified
from /root/reference by oracle/Makefile (target `refbridge`) -- with the
maintainer's HIPSpMVRef backend (spmv-vector-cache_amd/refbridge/: a subclass
of the reference's HardwareSpMV, registered through a factory branch) and a
driver that follows software/main.cpp:195-256: SparseMatrix::fromMemory on
the fixture files placed below 4 GiB, x = 1, y = 0, the reference's
markRowStarts for CMS, exec, then the reference's compareGolden against
golden.bin, printed as main.cpp's CSV.

CPU (this container): the program builds and runs the reference classes on
every f64 fixture -- rows/cols/nz as the reference loader reads them, the
factory branch taken -- and, with no GPU, reports the backend's no-device
status through statInt("error").  GPU: diffFromGolden == 0 on every fixture
(ORDERED, CMS on and off).  The GPU box has no reference tree: the GPU test
runs the binary built here (it travels with the tree) or skips."""
import os
import subprocess

import numpy as np
import pytest

import fixtures as fx

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "oracle", "_ref", "refbridge")
REF_TREE = "/root/reference/software/HardwareSpMV.cpp"


def _run(args, timeout=120):
    out = subprocess.run([BIN, "--dir", fx.MATRICES, *args], capture_output=True, text=True, timeout=timeout)
    lines = out.stdout.splitlines()
    hdr = next(l for l in lines if l.startswith("diffFromGolden,"))
    keys = hdr.rstrip(",").split(",")
    recs = [dict(zip(keys, l.rstrip(",").split(","))) for l in lines if l[:1].isdigit()]
    return out, recs


@pytest.mark.skipif(not os.path.exists(REF_TREE), reason="reference tree absent (GPU box)")
@pytest.mark.parametrize("cms", ["0", "1"])
def test_refbridge_runs_reference_classes_cpu(cms):
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "refbridge"], check=True, stdout=subprocess.DEVNULL)
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible: covered by the gpu test")
    out, recs = _run(["--cms", cms, *fx.F64_FIXTURES])
    assert out.returncode == 1, out.stdout + out.stderr  # exec() returned false: no device
    assert [r["matrix"] for r in recs] == fx.F64_FIXTURES
    for r in recs:
        rows, cols, colptr, rowind, _ = fx.load(r["matrix"])
        assert (int(r["rows"]), int(r["cols"]), int(r["nz"])) == (rows, cols, rowind.size), r
        assert r["accType"] == "HIPSpMV" and r["error"] == "6" and r["diffFromGolden"] != "0", r  # HIPSPMV_ERR_NO_DEVICE
    assert "no HIP device" in out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("cms", ["0", "1"])
def test_refbridge_reference_pipeline_gpu(gpu, cms):
    if not os.path.exists(BIN):
        pytest.skip("oracle/_ref/refbridge not built (needs the reference tree at build time)")
    out, recs = _run(["--cms", cms, "--reps", "2", *fx.F64_FIXTURES], timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert [r["matrix"] for r in recs] == fx.F64_FIXTURES
    for r in recs:
        assert r["diffFromGolden"] == "0" and r["error"] == "0" and r["accType"] == "HIPSpMV", r
        assert int(r["mode"]) == 1  # ORDERED: bit-identical to SoftwareSpMV, the reference's golden
    # the host golden the bridge compares with is A*1 (matrixutils.py:108-113)
    assert all(np.fromfile(os.path.join(fx.MATRICES, n, "golden.bin")).size == fx.load(n)[0]
               for n in fx.F64_FIXTURES)
