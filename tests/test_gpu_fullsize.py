"""BASELINE.json's two largest single-GPU configurations at full size:
C4 (2^24 x 2^24 stripe, 32 nnz/row, 537 M nonzeros) and C5 (R-MAT scale 24,
263 M nonzeros, longest row 238,554 entries).  Whole-matrix checks against the
C oracle's row-parallel CSR form (every row: ORDERED bit for bit, FAST within
the bound; the form is pinned to the CSC scatter by tests/test_oracle.py), and
size-independent ones:
a sample of rows (first, last, the longest, 2,000 random) is recomputed
sequentially in Python floats -- products rounded, then added in ascending
column order, exactly SoftwareSpMV's arithmetic (SoftwareSpMV.cpp:59-64) --
and ORDERED results must match those rows bit for bit, FAST results the
per-row bound of include/hipspmv.h; runs are deterministic.  With the values
read as u64 the checks are exact over the whole matrix: every kernel gives
the same bits, y is linear in x mod 2^64 and sum(y) equals a nonzero-wise
checksum.  Exercises the 64-bit entry offsets of every kernel and the hub-row
path of k_sell."""
import numpy as np
import pytest

import hipspmv as hs
import oracle

pytestmark = pytest.mark.gpu


def _sample(rowptr, n, k=2000):
    lens = np.diff(rowptr.astype(np.int64))
    rows = np.concatenate([[0, 1, n - 1, int(np.argmax(lens))], np.random.default_rng(7).integers(0, n, k)])
    return np.unique(rows)


def _sequential(rowptr, colind, vals, x, rows):
    want, absprod = [], []
    for r in rows:
        acc, ap = 0.0, 0.0
        for e in range(int(rowptr[r]), int(rowptr[r + 1])):
            p = float(vals[e]) * float(x[colind[e]])
            acc = acc + p
            ap = ap + abs(p)
        want.append(acc)
        absprod.append(ap)
    return np.array(want), np.array(absprod)


def _check(h, x, rows, want, absprod, lens, kernel, mode):
    h.set_kernel(kernel)  # the handle is shared by the module's tests: always (re)select
    y1 = h.exec(x, beta=0, mode=mode)
    y2 = h.exec(x, beta=0, mode=mode)
    assert y1.tobytes() == y2.tobytes(), (kernel, mode)  # deterministic
    got = y1[rows]
    if mode == hs.MODE_ORDERED:
        bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
        assert bad.size == 0, (kernel, h.kernel_name(mode), rows[bad[:5]])
    else:
        bound = 2.0 * np.maximum(lens[rows], 1) * 2.0 ** -53 * absprod + 1e-300
        assert np.all(np.abs(got - want) <= bound), (kernel, h.kernel_name(mode))
    return h.kernel_name(mode)


def _case(gen):
    n, rowptr, colind, vals = gen()
    x = hs.gen_vector(n, 3)
    rows = _sample(rowptr, n)
    want, absprod = _sequential(rowptr, colind, vals, x, rows)
    lens = np.diff(rowptr.astype(np.int64))
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    return h, x, rows, want, absprod, lens


@pytest.fixture(scope="module")
def c4_csr(gpu):
    return (1 << 24, *hs.gen_stripe_csr(0, 1 << 24, 1 << 24, 32))


@pytest.fixture(scope="module")
def c5_csr(gpu):
    return (1 << 24, *hs.gen_rmat_csr(24))


@pytest.fixture(scope="module")
def c3_csr(gpu):
    return (1 << 20, *hs.gen_stripe_csr(0, 1 << 20, 1 << 20, 32))


@pytest.fixture(scope="module")
def c4(c4_csr):
    case = _case(lambda: c4_csr)
    yield case
    case[0].close()


@pytest.fixture(scope="module")
def c5(c5_csr):
    case = _case(lambda: c5_csr)
    yield case
    case[0].close()


@pytest.mark.parametrize("kernel,mode", [("auto", hs.MODE_ORDERED), ("auto", hs.MODE_FAST),
                                         ("sell", hs.MODE_ORDERED), ("sell", hs.MODE_FAST),
                                         ("wcsr", hs.MODE_FAST)])
@pytest.mark.parametrize("which", ["c4", "c5"])
def test_full_size_sampled_rows(request, which, kernel, mode):
    h, x, rows, want, absprod, lens = request.getfixturevalue(which)
    _check(h, x, rows, want, absprod, lens, kernel, mode)


def _whole_oracle(rowptr, colind, vals, x):
    """y = A*x over every row by the oracle's row-parallel CSR restatement (oracle.c, 16 threads): each
    row summed sequentially in its CSR (ascending column) order, SoftwareSpMV's order -- bit-identical to
    the CSC scatter (tests/test_oracle.py::test_csr_rows_equal_csc_scatter)."""
    _, y = oracle.time_spmv_csr_f64_mt(rowptr, colind, vals, x, 1, 16)
    return y


def _whole_absprod(rowptr, colind, vals, x, chunk=1 << 25):
    """sum_e |a_e x[col_e]| per row (the FAST bound's scale), in row chunks."""
    n = rowptr.size - 1
    out = np.zeros(n)
    r0 = 0
    while r0 < n:
        r1 = min(n, int(np.searchsorted(rowptr, rowptr[r0] + chunk, side="right")) - 1)
        r1 = max(r1, r0 + 1)
        e0, e1 = int(rowptr[r0]), int(rowptr[r1])
        rows = np.repeat(np.arange(r1 - r0), np.diff(rowptr[r0:r1 + 1].astype(np.int64)))
        out[r0:r1] = np.bincount(rows, weights=np.abs(vals[e0:e1] * x[colind[e0:e1]]), minlength=r1 - r0)
        r0 = r1
    return out


@pytest.mark.parametrize("which", ["c4", "c5"])
def test_full_size_whole_matrix_against_oracle(request, which):
    """Every row of the full C4 / C5 matrix against the C oracle (the sampled-row checks
    above re-derive ~2,000 rows in Python): AUTO ORDERED bit-identical over the whole y, AUTO FAST
    within the per-row bound everywhere."""
    h, x, _, _, _, lens = request.getfixturevalue(which)
    n, rowptr, colind, vals = request.getfixturevalue(which + "_csr")
    want = _whole_oracle(rowptr, colind, vals, x)
    h.set_kernel("auto")
    y_o = h.exec(x, beta=0, mode=hs.MODE_ORDERED)
    bad = np.nonzero(y_o.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, (which, h.kernel_name(hs.MODE_ORDERED), bad[:5])
    y_f = h.exec(x, beta=0, mode=hs.MODE_FAST)
    bound = 2.0 * np.maximum(lens, 1) * 2.0 ** -53 * _whole_absprod(rowptr, colind, vals, x) + 1e-300
    over = np.nonzero(np.abs(y_f - want) > bound)[0]
    assert over.size == 0, (which, h.kernel_name(hs.MODE_FAST), over[:5])


def _checksum_u64(colind, vals, x, chunk=1 << 26):
    """sum_i y_i = sum_e a_e * x[col_e] (mod 2^64), in chunks."""
    s = np.uint64(0)
    for e0 in range(0, colind.size, chunk):
        s += np.sum(vals[e0:e0 + chunk] * x[colind[e0:e0 + chunk]], dtype=np.uint64)
    return int(s)


U64_KERNELS = {  # (kernel, mode); the C3 list includes the vector-cache kernels bench.py times
    "c3_csr": [("vcache", hs.MODE_ORDERED), ("vcache_split", hs.MODE_FAST), ("csr_lane", hs.MODE_ORDERED),
               ("csr_vector", hs.MODE_FAST), ("sell", hs.MODE_FAST)],
    # wide x (16 M columns, no vector-cache layout): every generic kernel by name
    "c4_csr": [("csr_lane", hs.MODE_ORDERED), ("csr_vector", hs.MODE_FAST), ("sell", hs.MODE_FAST),
               ("wgather", hs.MODE_ORDERED), ("wcsr", hs.MODE_FAST)],
    # wcsr: AUTO's FAST kernel for C5 (and its shards), by name on both
    "c5_csr": [("csr_lane", hs.MODE_ORDERED), ("csr_vector", hs.MODE_FAST), ("sell", hs.MODE_FAST),
               ("wcsr", hs.MODE_FAST)],
}


@pytest.mark.parametrize("which", ["c3_csr", "c4_csr", "c5_csr"])
def test_full_size_u64_exact_properties(request, which):
    """The same matrices with their 8-byte values read as u64 (the integer
    semiring, exact in every kernel and mode): every kernel/mode gives the
    same bits, y is linear in x mod 2^64 (A(x1 + x2) = Ax1 + Ax2), and
    sum(y) equals the nonzero-wise checksum sum_e a_e x[col_e] -- exact
    whole-matrix checks at full size, no sampling."""
    n, rowptr, colind, vals = request.getfixturevalue(which)
    a = vals.view(np.uint64)
    rng = np.random.default_rng(11)
    x1 = rng.integers(0, 2**64, n, dtype=np.uint64)
    x2 = rng.integers(0, 2**64, n, dtype=np.uint64)
    h = hs.Handle.from_csr(rowptr, colind, a, n, n)
    ran = set()
    try:
        ref = None
        with np.errstate(over="ignore"):
            for kernel, mode in U64_KERNELS[which]:
                h.set_kernel(kernel)
                y1 = h.exec(x1, beta=0, mode=mode)
                ran.add(h.kernel_name(mode))
                if ref is None:
                    ref = y1
                    y2 = h.exec(x2, beta=0, mode=mode)
                    y3 = h.exec(x1 + x2, beta=0, mode=mode)
                    assert np.array_equal(y3, y1 + y2), (which, kernel)  # linear mod 2^64
                    assert int(np.sum(y1, dtype=np.uint64)) == _checksum_u64(colind, a, x1), which
                else:
                    assert y1.tobytes() == ref.tobytes(), (which, kernel, h.kernel_name(mode))
        assert len(ran) == len(U64_KERNELS[which]), ran  # distinct kernels, none silently substituted
    finally:
        h.close()


@pytest.mark.parametrize("shard", [0, 7])
def test_c4_shard_auto_picks_wgather_split(c4_csr, shard):
    """C4 as the 8-GPU job runs it: a 2^21-row shard of the 2^24-column stripe matrix, created alone.
    AUTO's FAST kernel is wgather_split (bench.py's c4_shards block times it); sampled rows meet the
    FAST bound, deterministic.  With the values read as u64 the whole shard is exact: the same bits
    as the ordered wgather and sum(y) equal to the nonzero-wise checksum."""
    n, rowptr_all, colind_all, vals_all = c4_csr
    rows = n // 8
    r0 = shard * rows
    e0, e1 = int(rowptr_all[r0]), int(rowptr_all[r0 + rows])
    rowptr = (rowptr_all[r0:r0 + rows + 1] - rowptr_all[r0]).astype(np.uint32)
    colind, vals = colind_all[e0:e1], vals_all[e0:e1]
    x = hs.gen_vector(n, 3)
    sample = _sample(rowptr, rows, k=400)
    want, absprod = _sequential(rowptr, colind, vals, x, sample)
    lens = np.diff(rowptr.astype(np.int64))
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, n)
    try:
        assert h.kernel_name(hs.MODE_FAST) == "wgather_split", h.kernel_name(hs.MODE_FAST)
        assert h.stat("wgather_split_rows_per_block") == 16384 and h.stat("wgather_split_units") == 256
        _check(h, x, sample, want, absprod, lens, "auto", hs.MODE_FAST)
        y = h.exec(x, beta=0, mode=hs.MODE_FAST)  # every row of the shard against the C oracle
        bound = 2.0 * np.maximum(lens, 1) * 2.0 ** -53 * _whole_absprod(rowptr, colind, vals, x) + 1e-300
        assert np.all(np.abs(y - _whole_oracle(rowptr, colind, vals, x)) <= bound)
    finally:
        h.close()
    a = vals.view(np.uint64)
    xu = np.random.default_rng(13).integers(0, 2**64, n, dtype=np.uint64)
    hu = hs.Handle.from_csr(rowptr, colind, a, rows, n)
    try:
        hu.set_kernel("wgather_split")
        ys = hu.exec(xu, beta=0, mode=hs.MODE_FAST)
        hu.set_kernel("wgather")
        yw = hu.exec(xu, beta=0, mode=hs.MODE_ORDERED)
        assert ys.tobytes() == yw.tobytes()
        with np.errstate(over="ignore"):
            assert int(np.sum(ys, dtype=np.uint64)) == _checksum_u64(colind, a, xu)
    finally:
        hu.close()


@pytest.fixture(scope="module")
def c5_bounds(gpu):
    bounds, _ = hs.c5_partition(24, 8)  # bench.py's c5_shards partition (wcsr cost model)
    return bounds


@pytest.mark.parametrize("shard", [0, 3, 7])
def test_c5_shard_auto_picks_wcsr(c5_bounds, shard):
    """C5 as the 8-GPU job runs it: shards of the cost partition, each created alone.  AUTO's FAST
    kernel is wcsr on the hub-row shard 0, a middle shard and the short-row shard 7 (the bench's
    c5_shards block records it for all eight), and sampled rows meet the FAST bound."""
    r0, r1 = int(c5_bounds[shard]), int(c5_bounds[shard + 1])
    n = 1 << 24
    rowptr, colind, vals = hs.gen_rmat_rows(24, r0, r1, 16, 4)
    rows = r1 - r0
    x = hs.gen_vector(n, 3)
    sample = _sample(rowptr, rows, k=400)
    want, absprod = _sequential(rowptr, colind, vals, x, sample)
    lens = np.diff(rowptr.astype(np.int64))
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, n)
    try:
        assert h.kernel_name(hs.MODE_FAST) == "wcsr", (shard, h.kernel_name(hs.MODE_FAST))
        assert h.stat("wcsr_window_log2") == 20
        _check(h, x, sample, want, absprod, lens, "auto", hs.MODE_FAST)
    finally:
        h.close()
