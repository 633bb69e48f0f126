"""Pin the oracle's SparseMatrix restatements to the REFERENCE CODE itself.

oracle/_ref/libref_sparsematrix.so is the reference's own
software/SparseMatrix.cpp compiled unmodified where it lies (oracle/Makefile
target `ref`, harness oracle/ref_harness.cpp).  markRowStarts, maxAlive,
maxColSpan and clearRowMarkings of the oracle (oracle/oracle.c) and of the
product's host library (host/SparseMatrix.cpp via libspmvhost.so, the
statistics SoftwareSpMV and spmvbench report) must give the reference's exact
results -- marked index arrays bit for bit, the two
statistics equal -- on every fixture and on random matrices.  The GPU scans
(csrc/prep.hip, tests/test_gpu_prep.py) are checked against the oracle, so
this closes the chain to the reference for those statistics.

Only where /root/reference exists (this container; never the GPU box).
Inputs avoid the reference's undefined reads: maxColSpan reads
inds[colptr[c+1]-1] and inds[colptr[c]] for every column, which leaves the
array for an empty first or last column (SparseMatrix.cpp:113-115)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import fixtures as fx
import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/software/SparseMatrix.cpp"
LIB = os.path.join(REPO, "oracle", "_ref", "libref_sparsematrix.so")

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SRC), reason="reference tree absent (GPU box)")

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")


@pytest.fixture(scope="module")
def host():
    """The product's own SparseMatrix helpers (libspmvhost.so, host/SparseMatrix.cpp)."""
    import hipspmv as hs
    lib = hs.load_host()
    args = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p]
    lib.spmvhost_mark_row_starts.argtypes = args + [C.c_int, C.c_int]
    lib.spmvhost_mark_row_starts.restype = None
    lib.spmvhost_max_alive.argtypes = args
    lib.spmvhost_max_alive.restype = C.c_uint32
    lib.spmvhost_max_col_span.argtypes = args
    lib.spmvhost_max_col_span.restype = C.c_uint32
    lib.spmvhost_clear_row_markings.argtypes = args + [C.c_uint32]
    lib.spmvhost_clear_row_markings.restype = None
    return lib


@pytest.fixture(scope="module")
def ref():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True, stdout=subprocess.DEVNULL)
    lib = C.CDLL(LIB)
    args = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p]
    lib.ref_mark_row_starts.argtypes = args + [C.c_int, C.c_int]
    lib.ref_mark_row_starts.restype = None
    lib.ref_max_alive.argtypes = args
    lib.ref_max_alive.restype = C.c_uint32
    lib.ref_max_col_span.argtypes = args
    lib.ref_max_col_span.restype = C.c_uint32
    lib.ref_clear_row_markings.argtypes = args + [C.c_uint32]
    lib.ref_clear_row_markings.restype = None
    return lib


def _random_csc(seed, rows, cols, density, empty_inner_cols=True):
    rng = np.random.default_rng(seed)
    dense = rng.random((rows, cols)) < density
    dense[rng.integers(0, rows), 0] = True       # first and last column non-empty (see module doc)
    dense[rng.integers(0, rows), cols - 1] = True
    if empty_inner_cols and cols > 4:
        dense[:, rng.integers(1, cols - 1, size=cols // 8)] = False
    colptr = np.concatenate([[0], np.cumsum(dense.sum(0))]).astype(np.uint32)
    rowind = np.concatenate([np.nonzero(dense[:, c])[0] for c in range(cols)]).astype(np.uint32)
    return rows, cols, colptr, rowind


def _cases():
    out = []
    for name in fx.ALL_FIXTURES:
        rows, cols, colptr, rowind, _ = fx.load(name)
        if colptr[1] > colptr[0] and colptr[cols] > colptr[cols - 1]:
            out.append(pytest.param((rows, cols, colptr, rowind), id=name))
    for seed, (r, c, d) in enumerate([(50, 40, 0.1), (300, 17, 0.3), (7, 500, 0.05), (1000, 1000, 0.004),
                                      (33, 2, 0.5), (1, 9, 1.0)]):
        out.append(pytest.param(_random_csc(seed, r, c, d), id=f"rand{seed}_{r}x{c}"))
    return out


def _ref_call(ref, fn, case, inds, *extra):
    rows, cols, colptr, _ = case
    return getattr(ref, fn)(rows, cols, inds.size, np.ascontiguousarray(colptr, dtype=np.uint32), inds, *extra)


@pytest.mark.parametrize("case", _cases())
@pytest.mark.parametrize("reverse,shift", [(False, 31), (True, 30), (False, 30), (True, 31), (False, 29)])
def test_mark_row_starts_matches_reference(ref, host, case, reverse, shift):
    rows, cols, colptr, rowind = case
    want = rowind.copy()
    _ref_call(ref, "ref_mark_row_starts", case, want, int(reverse), shift)
    got = oracle.mark_row_starts(rowind, rows, reverse=reverse, shift=shift)
    assert got.tobytes() == want.tobytes()
    prod = rowind.copy()
    _ref_call(host, "spmvhost_mark_row_starts", case, prod, int(reverse), shift)
    assert prod.tobytes() == want.tobytes()


@pytest.mark.parametrize("case", _cases())
def test_max_alive_and_col_span_match_reference(ref, host, case):
    rows, cols, colptr, rowind = case
    ref_inds = rowind.copy()
    span = _ref_call(ref, "ref_max_col_span", case, rowind.copy())
    assert oracle.max_col_span(colptr, rowind) == span
    assert _ref_call(host, "spmvhost_max_col_span", case, rowind.copy()) == span
    want = _ref_call(ref, "ref_max_alive", case, ref_inds)
    prod = rowind.copy()
    assert _ref_call(host, "spmvhost_max_alive", case, prod) == want
    assert prod.tobytes() == ref_inds.tobytes()  # the product leaves the reference's marks
    _ref_call(host, "spmvhost_clear_row_markings", case, prod, 0x3FFFFFFF)
    assert prod.tobytes() == rowind.tobytes()
    mine = rowind.copy()
    got = int(oracle.lib().oracle_max_alive(rows, mine.size, mine))
    assert got == want
    # both leave the same marks behind (bits 31 and 30), and clearing them restores A
    assert mine.tobytes() == ref_inds.tobytes()
    _ref_call(ref, "ref_clear_row_markings", case, ref_inds, 0x3FFFFFFF)
    oracle.lib().oracle_clear_row_markings(mine.size, mine, 0x3FFFFFFF)
    assert mine.tobytes() == ref_inds.tobytes() == rowind.tobytes()


def test_marked_matrix_col_span_matches_reference(ref):
    # SoftwareSpMV::measurePreprocessingTimes calls maxColSpan on an unmarked A;
    # on a marked one the reference subtracts the raw words -- the oracle too
    rows, cols, colptr, rowind = _random_csc(11, 200, 60, 0.05)
    marked = oracle.mark_row_starts(oracle.mark_row_starts(rowind, rows), rows, reverse=True, shift=30)
    case = (rows, cols, colptr, marked)
    assert oracle.max_col_span(colptr, marked) == _ref_call(ref, "ref_max_col_span", case, marked.copy())
