"""GPU preprocessing scans (csrc/prep.hip via hipspmv_prep_stats /
hipspmv_mark_row_starts) vs the oracle's restatement of
SparseMatrix::maxAlive / maxColSpan / markRowStarts (SparseMatrix.cpp:52-119).
All integer: exact equality."""
import numpy as np
import pytest

import fixtures as fx
import hipspmv as hs
import oracle

pytestmark = pytest.mark.gpu


def _ragged_csc(rows, cols, seed, empty_cols=True):
    rng = np.random.default_rng(seed)
    counts = np.minimum(rng.integers(0, 9, cols), rows)
    if empty_cols:
        counts[:3] = 0  # leading empty columns
        counts[-3:] = 0  # trailing empty columns
        counts[cols // 2] = 0
    colptr = np.zeros(cols + 1, np.uint32)
    colptr[1:] = np.cumsum(counts)
    rowind = np.concatenate([np.sort(rng.choice(rows, c, replace=False)) for c in counts]).astype(np.uint32)
    return colptr, rowind


def _cases():
    for name in fx.ALL_FIXTURES:
        rows, cols, colptr, rowind, _ = fx.load(name)
        yield name, rows, colptr, rowind
    for seed, (rows, cols) in enumerate([(1000, 777), (50000, 20000), (3, 5000)]):
        colptr, rowind = _ragged_csc(rows, cols, seed)
        yield f"ragged{rows}x{cols}", rows, colptr, rowind


@pytest.mark.parametrize("case", list(range(len(fx.ALL_FIXTURES) + 3)))
def test_prep_stats_match_oracle(gpu, case):
    name, rows, colptr, rowind = list(_cases())[case]
    st = hs.prep_stats(colptr, rowind, rows)
    assert st["max_alive"] == oracle.max_alive(rowind, rows), name
    assert st["max_col_span"] == oracle.max_col_span(colptr, rowind), name
    assert st["max_alive_ns"] >= 0 and st["cms_ns"] >= 0


@pytest.mark.parametrize("reverse,shift", [(False, 31), (True, 30), (False, 30), (True, 31)])
def test_mark_row_starts_match_oracle(gpu, reverse, shift):
    for name, rows, colptr, rowind in _cases():
        got, ns = hs.mark_row_starts(rowind, rows, reverse=reverse, shift=shift)
        want = oracle.mark_row_starts(rowind, rows, reverse=reverse, shift=shift)
        assert np.array_equal(got, want), (name, reverse, shift)
        assert ns >= 0


def test_prep_stats_large_stripe(gpu):
    # C3 shape: 2^20 x 2^20, 32 nnz/row, in CSC as SparseMatrix holds it
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    colptr, rowind, _ = oracle.csr2csc(n, n, rowptr, colind, vals)
    st = hs.prep_stats(colptr, rowind, n)
    assert st["max_alive"] == oracle.max_alive(rowind, n)
    assert st["max_col_span"] == oracle.max_col_span(colptr, rowind)


def test_prep_marked_input_is_masked(gpu):
    # marks already present (main.cpp:228-229 marks A before the backend runs)
    rows, cols, colptr, rowind, _ = fx.load("circuit204")
    marked = oracle.mark_row_starts(rowind, rows)
    st = hs.prep_stats(colptr, marked, rows)
    assert st["max_alive"] == oracle.max_alive(rowind, rows)
    assert st["max_col_span"] == oracle.max_col_span(colptr, rowind)


def test_prep_invalid_row(gpu):
    colptr = np.array([0, 2], np.uint32)
    rowind = np.array([0, 9], np.uint32)
    with pytest.raises(hs.HipSpMVError) as e:
        hs.prep_stats(colptr, rowind, 4)
    assert e.value.status == 2  # HIPSPMV_ERR_INVALID_MATRIX
    with pytest.raises(hs.HipSpMVError):
        hs.mark_row_starts(rowind, 4)


def test_prep_empty_matrix(gpu):
    st = hs.prep_stats(np.zeros(6, np.uint32), np.zeros(0, np.uint32), 4)
    assert st["max_alive"] == 0 and st["max_col_span"] == 0
    out, _ = hs.mark_row_starts(np.zeros(0, np.uint32), 4)
    assert out.size == 0
