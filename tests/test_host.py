"""CPU tests of the product host library (libspmvhost.so): the restated
plugin surface, loaders, generators, csr2csc and row partitioning."""
import os
import subprocess
import sys

import numpy as np
import pytest

import fixtures as fx
import hipspmv as hs
import oracle

SPMVBENCH = os.path.join(hs.LIB_DIR, "spmvbench")


@pytest.mark.parametrize("name", fx.ALL_FIXTURES)
def test_loader_matches_numpy_reader(name):
    rows, cols, colptr, rowind, vals = hs.load_matrix(fx.MATRICES, name)
    r2, c2, cp2, ri2, v2 = fx.load(name)
    assert (rows, cols) == (r2, c2)
    assert np.array_equal(colptr, cp2) and np.array_equal(rowind, ri2) and vals.tobytes() == v2.tobytes()
    assert vals.dtype == v2.dtype


def test_matrix_market_conversion_is_byte_identical(tmp_path):
    # matrices/mtx/circuit204.mtx -> the reference's circuit204/*.bin, byte for byte,
    # including the Zynq base addresses in -meta.bin and golden.bin = A*1
    hs.convert_mtx(os.path.join(fx.MATRICES, "mtx", "circuit204.mtx"), str(tmp_path), "circuit204")
    for suffix in ("-meta.bin", "-indptr.bin", "-inds.bin", "-data.bin"):
        a = open(os.path.join(tmp_path, "circuit204", "circuit204" + suffix), "rb").read()
        b = open(os.path.join(fx.MATRICES, "circuit204", "circuit204" + suffix), "rb").read()
        assert a == b, suffix
    a = open(os.path.join(tmp_path, "circuit204", "golden.bin"), "rb").read()
    assert a == open(os.path.join(fx.MATRICES, "circuit204", "golden.bin"), "rb").read()


def _run_sw(names):
    out = subprocess.run([SPMVBENCH, "--dir", fx.MATRICES, "--confs", "sw", "--cms", "0", *names],
                         capture_output=True, text=True, check=True).stdout.splitlines()
    hdr_i = next(i for i, l in enumerate(out) if l.startswith("rows,"))
    keys = out[hdr_i].rstrip(",").split(",")
    rows = [dict(zip(keys, l.rstrip(",").split(","))) for l in out[hdr_i + 1:] if l and l[0].isdigit()]
    return rows


def test_softwarespmv_preprocessing_stats_match_oracle():
    # SoftwareSpMV::measurePreprocessingTimes (SoftwareSpMV.cpp:72-94) vs oracle
    names = ["circuit204", "row64k", "i64", "dia64-uint64", "rowvec64-uint64"]
    for rec in _run_sw(names):
        rows, cols, colptr, rowind, vals = fx.load(rec["matrix"])
        ind = rowind.copy()
        assert int(rec["maxColSpan"]) == oracle.lib().oracle_max_col_span(cols, colptr, ind)
        assert int(rec["maxAlive"]) == oracle.lib().oracle_max_alive(rows, rowind.size, ind)
        assert (int(rec["rows"]), int(rec["cols"]), int(rec["nz"])) == (rows, cols, rowind.size)


def test_mark_row_starts_matches_oracle():
    rows, cols, colptr, rowind, vals = fx.load("circuit204")
    a = rowind.copy()
    oracle.lib().oracle_mark_row_starts(rows, a.size, a, 0, 31)
    first = {}
    for e, r in enumerate(rowind):
        first.setdefault(int(r), e)
    marked = set(np.nonzero(a & np.uint32(1 << 31))[0].tolist())
    assert marked == set(first.values())


def test_stripe_generator_properties():
    n, k = 1 << 14, 32
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, k)
    assert np.array_equal(rowptr, np.arange(n + 1, dtype=np.uint32) * k)
    c = colind.reshape(n, k).astype(np.int64)
    w = n // k
    assert np.all(c // w == np.arange(k)[None, :])   # one column per stripe, sorted
    assert np.all((vals >= -1) & (vals < 1))
    # a shard generates exactly the rows of the whole matrix
    rp2, ci2, v2 = hs.gen_stripe_csr(777, 100, n, k)
    assert np.array_equal(ci2, colind[777 * k:877 * k]) and np.array_equal(v2, vals[777 * k:877 * k])


def test_splitmix64_reference_values():
    # splitmix64 seeded with 0: first outputs (Vigna's reference implementation)
    lib = hs.load_host()
    assert lib.spmvhost_splitmix64_at(0, 0) == 0xE220A8397B1DCDAF
    assert lib.spmvhost_splitmix64_at(0, 1) == 0x6E789E6AA1B965F4


def test_rmat_generator_is_valid_csr():
    rowptr, colind, vals = hs.gen_rmat_csr(10, 16, seed=4)
    n = 1 << 10
    assert rowptr[0] == 0 and rowptr[-1] == colind.size and np.all(np.diff(rowptr.astype(np.int64)) >= 0)
    for r in range(n):
        seg = colind[rowptr[r]:rowptr[r + 1]].astype(np.int64)
        assert np.all(np.diff(seg) > 0)  # duplicates summed, ascending
    lens = np.diff(rowptr.astype(np.int64))
    assert lens.max() > 8 * lens.mean()  # skewed (power law)


@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_partition_rows_balanced(parts):
    rowptr, colind, vals = hs.gen_rmat_csr(12, 16, seed=4)
    b = hs.partition_rows(rowptr, parts).astype(np.int64)
    assert b[0] == 0 and b[-1] == rowptr.size - 1 and np.all(np.diff(b) >= 0)
    assert np.all(b[1:-1] % 64 == 0)  # shard starts at multiples of HIPSPMV_SHARD_ALIGN
    nnz = rowptr[b[1:]].astype(np.int64) - rowptr[b[:-1]].astype(np.int64)
    assert nnz.sum() == colind.size
    lens = np.diff(rowptr.astype(np.int64))
    slack = np.sort(lens)[-33:].sum()  # the snap moves a cut by at most 32 rows each way
    assert nnz.max() <= colind.size / parts + 2 * slack + 1


def test_product_csr2csc_equals_oracle():
    rowptr, colind, vals = hs.gen_rmat_csr(9, 8, seed=9)
    n = 1 << 9
    a = hs.csr2csc(n, n, rowptr, colind, vals)
    b = oracle.csr2csc(n, n, rowptr, colind, vals)
    for u, v in zip(a, b):
        assert u.tobytes() == v.tobytes()


def test_rmat_row_ranges_concatenate_to_the_whole_matrix():
    scale = 13
    rowptr, colind, vals = hs.gen_rmat_csr(scale, 16, 4)
    counts = hs.gen_rmat_row_counts(scale, 16, 4)
    assert int(counts.sum(dtype=np.uint64)) == 16 << scale
    assert np.all(np.diff(rowptr.astype(np.int64)) <= counts)  # duplicates only shrink rows
    for parts in (1, 3, 8):
        b = hs.partition_row_counts(counts, parts)
        assert b[0] == 0 and b[-1] == 1 << scale and np.all(np.diff(b.astype(np.int64)) >= 0)
        assert np.all(b[1:-1] % 64 == 0)
        for p in range(parts):
            r0, r1 = int(b[p]), int(b[p + 1])
            rp, ci, v = hs.gen_rmat_rows(scale, r0, r1, 16, 4)
            e0, e1 = int(rowptr[r0]), int(rowptr[r1])
            assert np.array_equal(rp, rowptr[r0:r1 + 1] - rowptr[r0])
            assert np.array_equal(ci, colind[e0:e1]) and v.tobytes() == vals[e0:e1].tobytes()
        if parts == 8:  # nnz balance of the count-based split
            share = np.diff(rowptr[b.astype(np.int64)].astype(np.int64)) / rowptr[-1]
            assert share.max() < 1.5 / parts


def test_generators_independent_of_thread_count(monkeypatch):
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); import hipspmv as hs, hashlib; "
            "a = hs.gen_rmat_csr(12); b = hs.gen_stripe_csr(5, 3000, 1 << 20); "
            "print(hashlib.sha256(b''.join(x.tobytes() for x in a + b)).hexdigest())") % hs.PKG_DIR
    outs = set()
    for t in ("1", "3", "8"):
        env = dict(os.environ, SPMV_THREADS=t)
        outs.add(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                check=True).stdout)
    assert len(outs) == 1


def _scipy_csc(name):
    import scipy.sparse as sp
    rows, cols, colptr, rowind, vals = fx.load(name)
    return sp.csc_matrix((vals, rowind, colptr), shape=(rows, cols)), (rows, cols, colptr, rowind, vals)


def _ref_row_len_histogram(matrix):
    # matrices/matrixutils.py:116-126 restated (Python 3): note the loop bound
    csr = matrix.tocsr()
    h = {}
    for j in range(1, csr.shape[1]):
        n = int(csr.indptr[j] - csr.indptr[j - 1])
        h[n] = h.get(n, 0) + 1
    return h


def _ref_permute_longest_row_first(matrix):
    # matrices/matrixutils.py:140-158 restated (Python 3, scipy as the reference)
    import scipy.sparse as sp
    csr = matrix.tocsr()
    csr.sort_indices()
    lens = sorted(zip([int(csr.indptr[i + 1] - csr.indptr[i]) for i in range(csr.shape[0])],
                      range(csr.shape[0])), reverse=True)
    perm = [x[1] for x in lens]
    P = sp.coo_matrix(([1 for _ in perm], (range(len(perm)), perm)))
    return perm, (P * csr).tocsc()


@pytest.mark.parametrize("name", ["circuit204", "i1k", "row64k", "dia64-uint64", "rowvec64-uint64"])
def test_row_len_histogram_matches_matrixutils(name):
    A, (rows, cols, colptr, rowind, vals) = _scipy_csc(name)
    assert hs.row_len_histogram(colptr, rowind, rows) == _ref_row_len_histogram(A)


@pytest.mark.parametrize("name", ["circuit204", "i64", "rowvec64-uint64", "dia64-uint64"])
def test_permute_longest_row_first_matches_matrixutils(name):
    A, (rows, cols, colptr, rowind, vals) = _scipy_csc(name)
    perm, cp, ri, v = hs.permute_longest_row_first(colptr, rowind, vals, rows)
    ref_perm, B = _ref_permute_longest_row_first(A.astype(np.float64))
    assert perm.tolist() == ref_perm
    B.sort_indices()
    assert np.array_equal(cp, B.indptr) and np.array_equal(ri, B.indices)
    if vals.dtype == np.float64:
        assert v.tobytes() == B.data.astype(np.float64).tobytes()
    else:
        assert np.array_equal(v, B.data.astype(np.uint64))


def test_convert_mtx_permuted(tmp_path):
    import scipy.io as sio
    mtx = os.path.join(fx.MATRICES, "mtx", "circuit204.mtx")
    hs.convert_mtx(mtx, str(tmp_path), "c204p", golden=True, permute=True)
    rows, cols, colptr, rowind, vals = hs.load_matrix(str(tmp_path), "c204p")
    _, B = _ref_permute_longest_row_first(sio.mmread(mtx).tocsc())
    B.sort_indices()
    assert np.array_equal(colptr, B.indptr) and np.array_equal(rowind, B.indices)
    assert vals.tobytes() == B.data.tobytes()
    # golden of the permuted matrix = the reference golden permuted
    g = np.fromfile(os.path.join(str(tmp_path), "c204p", "golden.bin"), dtype=np.float64)
    perm, *_ = hs.permute_longest_row_first(*fx.load("circuit204")[2:5], 1020)
    assert g.tobytes() == fx.golden("circuit204")[perm].tobytes()
