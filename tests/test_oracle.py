"""Pin the CPU oracle (oracle/oracle.c) to the reference's own data before
trusting it: every golden.bin, the frontend known-answer tests, csr2csc."""
import numpy as np
import pytest

import fixtures as fx
import oracle


@pytest.mark.parametrize("name", fx.F64_FIXTURES)
def test_oracle_matches_reference_golden(name):
    # golden.bin = A*ones written by matrices/matrixutils.py:108-113
    rows, cols, colptr, rowind, vals = fx.load(name)
    y = oracle.spmv_csc(colptr, rowind, vals, np.ones(cols), rows=rows)
    g = fx.golden(name)
    assert y.tobytes() == g.tobytes()


def test_kat_identity_64_u64():
    # chisel/tests/TestSpMVFrontend.scala:121-143: identity 64x64, x = 1..64 -> sum y = 2080
    rows, cols, colptr, rowind, vals = fx.load("i64-uint64")
    y = oracle.spmv_csc(colptr, rowind, vals, np.arange(1, 65, dtype=np.uint64), rows=rows)
    assert int(y.sum()) == 2080 and np.array_equal(y, np.arange(1, 65, dtype=np.uint64))


def test_kat_rowvector_64_u64():
    # TestSpMVFrontend.scala:148-182: 1x64 row vector, x = 1..64 -> y0 = 2080
    rows, cols, colptr, rowind, vals = fx.load("rowvec64-uint64")
    y = oracle.spmv_csc(colptr, rowind, vals, np.arange(1, 65, dtype=np.uint64), rows=rows)
    assert int(y[0]) == 2080 and int(y[1:].sum()) == 0


def test_u64_fixture_values():
    # SURVEY Appendix A values for the integer fixtures
    r, c, cp, ri, v = fx.load("dia64-uint64")
    assert int(oracle.spmv_csc(cp, ri, v, np.ones(c, np.uint64), rows=r).sum()) == 2016
    assert int(oracle.spmv_csc(cp, ri, v, np.arange(1, c + 1, dtype=np.uint64), rows=r).sum()) == 87360
    r, c, cp, ri, v = fx.load("circuit204-uint64")
    y1 = oracle.spmv_csc(cp, ri, v, np.ones(c, np.uint64), rows=r)
    assert list(y1[:4]) == [3, 6, 10, 14] and int(y1.sum()) == 5883
    y2 = oracle.spmv_csc(cp, ri, v, np.arange(1, c + 1, dtype=np.uint64), rows=r)
    assert list(y2[:4]) == [157, 595, 875, 741] and int(y2.sum()) == 2486898


def test_u64_wraps_mod_2_64():
    # StagedUIntOp(64): product and sum truncated to 64 bits (SemiringOp.scala:74-92)
    colptr = np.array([0, 2, 3], np.uint32)
    rowind = np.array([0, 0, 1], np.uint32)
    vals = np.array([2**63 + 5, 2**62, 2**64 - 1], np.uint64)
    x = np.array([3, 7], np.uint64)
    y = oracle.spmv_csc(colptr, rowind, vals, x, rows=2)
    m = 2**64
    assert int(y[0]) == (((2**63 + 5) * 3) % m + (2**62 * 3) % m) % m
    assert int(y[1]) == ((2**64 - 1) * 7) % m


def test_oracle_u64_agrees_with_python_ints():
    rng = np.random.default_rng(3)
    rows, cols = 37, 29
    dense = (rng.random((rows, cols)) < 0.2)
    colptr = np.concatenate([[0], np.cumsum(dense.sum(0))]).astype(np.uint32)
    rowind = np.concatenate([np.nonzero(dense[:, c])[0] for c in range(cols)]).astype(np.uint32)
    vals = rng.integers(0, 2**64, size=rowind.size, dtype=np.uint64)
    x = rng.integers(0, 2**64, size=cols, dtype=np.uint64)
    y = oracle.spmv_csc(colptr, rowind, vals, x, rows=rows)
    ref = [0] * rows
    for c in range(cols):
        for e in range(colptr[c], colptr[c + 1]):
            ref[rowind[e]] = (ref[rowind[e]] + int(vals[e]) * int(x[c])) % 2**64
    assert [int(v) for v in y] == ref


def test_oracle_accumulates_into_y():
    # SoftwareSpMV.cpp:62 is y += ...: a second exec doubles y (x = ones)
    rows, cols, colptr, rowind, vals = fx.load("circuit204")
    y = oracle.spmv_csc(colptr, rowind, vals, np.ones(cols), rows=rows)
    y2 = oracle.spmv_csc(colptr, rowind, vals, np.ones(cols), y=y.copy(), rows=rows)
    ref = y.copy()
    oracle.spmv_csc(colptr, rowind, vals, np.ones(cols), y=ref, rows=rows)
    assert np.array_equal(y2, ref)


@pytest.mark.parametrize("name", fx.ALL_FIXTURES)
def test_csr2csc_roundtrip(name):
    rows, cols, colptr, rowind, vals = fx.load(name)
    # CSC -> CSR (transpose roles), then back: identical arrays (stable sort)
    rowptr, colind, rvals = oracle.csr2csc(cols, rows, colptr, rowind, vals)
    cp2, ri2, v2 = oracle.csr2csc(rows, cols, rowptr, colind, rvals)
    assert np.array_equal(cp2, colptr) and np.array_equal(ri2, rowind) and v2.tobytes() == vals.tobytes()
    # CSR rows come out with ascending column ids
    for r in range(min(rows, 2000)):
        seg = colind[rowptr[r]:rowptr[r + 1]]
        assert np.all(np.diff(seg.astype(np.int64)) >= 0)


def test_dense_crosscheck_circuit204():
    rows, cols, colptr, rowind, vals = fx.load("circuit204")
    A = fx.csc_to_dense(rows, cols, colptr, rowind, vals)
    x = np.random.default_rng(1).uniform(-1, 1, cols)
    y = oracle.spmv_csc(colptr, rowind, vals, x, rows=rows)
    np.testing.assert_allclose(y, A @ x, rtol=1e-12, atol=1e-14)


def test_csr_rows_equal_csc_scatter():
    # the oracle's row-parallel CSR form (oracle_time_spmv_csr_f64_mt: each row summed from +0.0 in its
    # CSR order) gives SoftwareSpMV's CSC scatter bits on every row -- empty rows, a full-width row,
    # repeated columns -- so the full-size GPU tests may use it as the whole-matrix oracle
    rng = np.random.default_rng(21)
    rows, cols = 30011, 5003
    lens = rng.integers(0, 40, rows)
    lens[rng.integers(0, rows, rows // 5)] = 0
    per_row = [np.sort(rng.integers(0, cols, n)) for n in lens]  # sorted, with repeats
    per_row[17] = np.arange(cols)
    lens = np.array([c.size for c in per_row])
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate(per_row).astype(np.uint32)
    vals = rng.uniform(-1, 1, colind.size)
    x = rng.uniform(-1, 1, cols)
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    want = oracle.spmv_csc(colptr, rowind, cvals, x, rows=rows)
    for nt in (1, 7, 16):
        _, y = oracle.time_spmv_csr_f64_mt(rowptr, colind, vals, x, 1, nt)
        assert y.tobytes() == want.tobytes(), nt
