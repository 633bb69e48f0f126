"""GPU parity: the HIP kernels through the C ABI vs the CPU oracle.

Ordered kernels (vcache, csr_lane) and every u64 run must be bit-identical
to SoftwareSpMV (oracle.spmv_csc); the fast f64 kernel (csr_vector) must meet
the per-row bound of include/hipspmv.h:
    |y - y_ref| <= 2*len*2^-53 * (sum_j |a_ij x_j| + |y_in|)  (+ tiny abs slack)
"""
import os

import numpy as np
import pytest

import fixtures as fx
import hipspmv as hs
import oracle

pytestmark = pytest.mark.gpu

ORDERED_KERNELS = ["vcache", "csr_lane", "sell"]


def _fast_bound(rowptr_len, absprod, yin):
    u = 2.0 ** -53
    return 2.0 * np.maximum(rowptr_len, 1) * u * (absprod + np.abs(yin)) + 1e-300


def _csr_stats(rows, cols, colptr, rowind, vals, x):
    """per-row length and sum|a_ij x_j| (for the fast-mode bound)"""
    lens = np.bincount(rowind, minlength=rows)
    absprod = np.zeros(rows)
    np.add.at(absprod, rowind, np.abs(vals.astype(np.float64) * np.repeat(x, np.diff(colptr.astype(np.int64)))))
    return lens, absprod


def _check(name, rows, cols, colptr, rowind, vals, x, kernel, beta, mode=hs.MODE_ORDERED, y0=None):
    h = hs.Handle.from_csc(colptr, rowind, vals, rows, cols)
    if (kernel == "vcache" and not h.stat("vcache_eligible")) or \
            (kernel == "vcache_split" and not h.stat("vcache_split_eligible")) or \
            (kernel == "vcache_split4" and not h.stat("vcache_split4_eligible")):
        pytest.skip("vcache not eligible")
    try:
        h.set_kernel(kernel)
    except hs.HipSpMVError as e:  # the four-part layouts are placed on selection, and may not fit
        if kernel in ("vcache_split4", "vcache_flow") and e.status == 5:
            pytest.skip(f"{kernel}: layout not placeable for this matrix")
        raise
    npdt = vals.dtype
    if y0 is None:
        y0 = (np.random.default_rng(11).uniform(-1, 1, rows) if npdt == np.float64
              else np.random.default_rng(11).integers(0, 2**64, rows, dtype=np.uint64))
    y_ref = oracle.spmv_csc(colptr, rowind, vals, x, y=(y0.copy() if beta else np.zeros(rows, npdt)), rows=rows)
    y = h.exec(x, y0.copy(), beta=beta, mode=mode)
    if npdt == np.uint64 or kernel in ORDERED_KERNELS:
        if y.tobytes() != y_ref.tobytes():
            bad = np.nonzero(y.view(np.uint64) != y_ref.view(np.uint64))[0]
            pytest.fail(f"{name}/{kernel}/beta{beta}: {bad.size} rows differ, first {bad[:5]} "
                        f"got {y[bad[:3]]} want {y_ref[bad[:3]]}")
    else:
        lens, absprod = _csr_stats(rows, cols, colptr, rowind, vals, x)
        bound = _fast_bound(lens, absprod, y0 if beta else np.zeros(rows))
        err = np.abs(y - y_ref)
        assert np.all(err <= bound), f"{name}: max err/bound {np.max(err / bound)}"
    return h, y


@pytest.mark.parametrize("name", fx.ALL_FIXTURES)
@pytest.mark.parametrize("kernel", ["vcache", "csr_lane", "csr_vector", "vcache_split", "sell", "wcsr",
                                    "vcache_split4", "vcache_flow"])
@pytest.mark.parametrize("beta", [0, 1])
def test_fixtures(gpu, name, kernel, beta):
    rows, cols, colptr, rowind, vals = fx.load(name)
    for xname, x in fx.x_variants(name, cols).items():
        mode = hs.MODE_ORDERED if kernel in ORDERED_KERNELS else hs.MODE_FAST
        _check(f"{name}[{xname}]", rows, cols, colptr, rowind, vals, x, kernel, beta, mode)


def _tile_columns(cols, colptr, rowind, vals, k):
    """[A A ... A] (k copies side by side): the reference fixture widened until
    the column-part geometries apply, rows and their column order intact"""
    nnz = rowind.size
    cp = np.concatenate([colptr[:-1].astype(np.int64) + j * nnz for j in range(k)] + [[k * nnz]]).astype(np.uint32)
    return k * cols, cp, np.tile(rowind, k), np.tile(vals, k)


@pytest.mark.parametrize("name", ["circuit204", "circuit204-uint64"])
@pytest.mark.parametrize("kernel", ["vcache_split", "vcache_split4", "vcache_flow"])
@pytest.mark.parametrize("beta", [0, 1])
def test_tiled_fixture_column_parts(gpu, name, kernel, beta):
    # the headline FAST kernels on a reference-held matrix: circuit204 tiled to
    # 12 x 1020 = 12,240 columns (three / four column parts) against the oracle
    rows, cols, colptr, rowind, vals = fx.load(name)
    k = -(-12001 // cols)
    tcols, tcp, tri, tv = _tile_columns(cols, colptr, rowind, vals, k)
    h = hs.Handle.from_csc(tcp, tri, tv, rows, tcols)
    if kernel == "vcache_split":
        assert h.stat("vcache_split_eligible"), (name, tcols)  # the product FAST kernel runs it
    elif kernel == "vcache_flow":
        pass  # (placed on selection in _check; circuit204's rows are short: it fits)
    elif not h.stat("vcache_split4_eligible"):
        # k_vquad holds a segment in registers (<= 1664 entries); circuit204's 1020 rows
        # put ~2 x 5.9 k entries into each 1984-column panel
        h.close()
        pytest.skip("k_vquad: segments past its register window")
    h.close()
    for xname, x in fx.x_variants(name, tcols).items():
        _, y = _check(f"{name}x{k}[{xname}]", rows, tcols, tcp, tri, tv, x, kernel, beta, hs.MODE_FAST)


@pytest.mark.parametrize("name", fx.F64_FIXTURES)
def test_reference_golden_bin_exact(gpu, name):
    # HIPSpMV ordered == reference golden.bin (A*1), the reference's own compareGolden
    rows, cols, colptr, rowind, vals = fx.load(name)
    h = hs.Handle.from_csc(colptr, rowind, vals, rows, cols)
    y = h.exec(np.ones(cols), beta=0, mode=hs.MODE_ORDERED)
    assert y.tobytes() == fx.golden(name).tobytes(), h.kernel_name(hs.MODE_ORDERED)


def _random_csc(rows, cols, density, rng, dtype=np.float64, empty_rows=True, long_rows=(), dup=False):
    dense = rng.random((rows, cols)) < density
    if empty_rows:
        dense[rng.integers(0, rows, rows // 7)] = False
    for r in long_rows:
        dense[r, :] = True
    colptr = np.concatenate([[0], np.cumsum(dense.sum(0))]).astype(np.uint32)
    rowind = np.concatenate([np.nonzero(dense[:, c])[0] for c in range(cols)]).astype(np.uint32)
    if dup:  # repeat ~5% of the entries right after themselves in their column (SoftwareSpMV adds both, in order)
        col_of = np.repeat(np.arange(cols), dense.sum(0))
        k = 1 + (rng.random(rowind.size) < 0.05).astype(np.int64)
        rowind, col_of = np.repeat(rowind, k), np.repeat(col_of, k)
        colptr = np.concatenate([[0], np.cumsum(np.bincount(col_of, minlength=cols))]).astype(np.uint32)
    if dtype == np.float64:
        vals = rng.uniform(-1, 1, rowind.size)
    else:
        vals = rng.integers(0, 2**64, rowind.size, dtype=np.uint64)
    return colptr, rowind, vals


# (700, 20001): odd columns over 6 panels of the split geometry (2 per part, the last
# panel patched); (900, 14001): 4 panels, column parts of 1, 1 and 2 (vc_part_first);
# (1, 40001), (64, 12001), (4097, 12001): ragged shapes wide enough for the split
# geometry (its irregular coverage) -- one row, one row per lane group,
# a block boundary one row past 4096, each with a full-width row
@pytest.mark.parametrize("shape", [(1, 1), (1, 300), (300, 1), (257, 1000), (5000, 333), (3000, 20000),
                                   (700, 20001), (900, 14001), (1, 40001), (64, 12001), (4097, 12001)])
@pytest.mark.parametrize("kernel", ["vcache", "csr_lane", "csr_vector", "vcache_split", "sell", "wcsr",
                                    "vcache_split4", "vcache_flow"])
def test_random_ragged(gpu, shape, kernel):
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    rows, cols = shape
    dens = min(1.0, 40.0 / cols)
    colptr, rowind, vals = _random_csc(rows, cols, dens, rng, long_rows=[rows // 2] if rows > 2 else [])
    x = rng.uniform(-1, 1, cols)
    mode = hs.MODE_ORDERED if kernel in ORDERED_KERNELS else hs.MODE_FAST
    for beta in (0, 1):
        _check(f"rand{shape}", rows, cols, colptr, rowind, vals, x, kernel, beta, mode)


@pytest.mark.parametrize("kernel", ["vcache", "csr_lane", "csr_vector", "vcache_split", "sell", "wcsr",
                                    "vcache_split4", "vcache_flow"])
def test_random_u64_wraparound(gpu, kernel):
    rng = np.random.default_rng(5)
    rows, cols = 4000, 9000
    colptr, rowind, vals = _random_csc(rows, cols, 0.004, rng, dtype=np.uint64, long_rows=[17])
    x = rng.integers(0, 2**64, cols, dtype=np.uint64)
    for beta in (0, 1):
        _check("u64", rows, cols, colptr, rowind, vals, x, kernel, beta, hs.MODE_FAST)


@pytest.mark.parametrize("kernel", ["vcache", "csr_lane", "csr_vector", "vcache_split", "sell", "wcsr",
                                    "vcache_split4", "vcache_flow"])
def test_random_duplicates(gpu, kernel):
    # repeated (row, col) entries (5 % of a ragged matrix with a full-width row):
    # ORDERED kernels add each copy in CSC order, bit for bit; FAST within the bound
    # 20001 columns: enough panels for the three-part split geometry (6), odd width
    rng = np.random.default_rng(11)
    rows, cols = 2000, 20001
    colptr, rowind, vals = _random_csc(rows, cols, 0.0015, rng, long_rows=[77], dup=True)
    assert np.any(np.diff(rowind.astype(np.int64)) == 0)  # some entry is repeated
    x = rng.uniform(-1, 1, cols)
    mode = hs.MODE_ORDERED if kernel in ORDERED_KERNELS else hs.MODE_FAST
    for beta in (0, 1):
        _check("dup", rows, cols, colptr, rowind, vals, x, kernel, beta, mode)


@pytest.mark.parametrize("dtype", [np.float64, np.uint64])
def test_wcsr_wide_windows(gpu, dtype):
    # wcsr cuts rows at 2^20-column windows: a wide, skewed matrix (rows spanning every window, a
    # full-width row, empty rows, an odd column count) -- FAST within the bound and identical bits
    # on every run; u64 exact; the segment count matches a CPU recount
    rng = np.random.default_rng(21)
    rows, cols = 3000, (1 << 21) + 13
    want = rng.zipf(1.6, rows).clip(0, 40000)
    want[rng.integers(0, rows, 300)] = 0
    want[5] = 60000
    per_row = [np.unique(rng.integers(0, cols, int(n))) for n in want]  # sorted, distinct
    lens = np.array([c.size for c in per_row], np.int64)
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate(per_row).astype(np.uint32)
    if dtype == np.float64:
        vals, x = rng.uniform(-1, 1, colind.size), rng.uniform(-1, 1, cols)
    else:
        vals = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
        x = rng.integers(0, 2**64, cols, dtype=np.uint64)
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.kernel_name(hs.MODE_FAST) == "wcsr"  # AUTO: x wider than the L2s, rows windowable
    h.set_kernel("wcsr")
    row_of = np.repeat(np.arange(rows), lens)
    lw = h.stat("wcsr_window_log2")
    # segments: each row's run in one window, cut into pieces of <= 256 entries (the layout's cap)
    _, runs = np.unique(row_of.astype(np.int64) * 4096 + (colind >> lw), return_counts=True)
    assert h.stat("wcsr_segments") == int(np.sum((runs + 255) // 256))
    y0 = (rng.uniform(-1, 1, rows) if dtype == np.float64 else rng.integers(0, 2**64, rows, dtype=np.uint64))
    for beta in (0, 1):
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else np.zeros(rows, dtype)), rows=rows)
        ys = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(2)]
        assert ys[0].tobytes() == ys[1].tobytes()
        if dtype == np.uint64:
            assert ys[0].tobytes() == y_ref.tobytes()
        else:
            absprod = np.zeros(rows)
            np.add.at(absprod, row_of, np.abs(vals * x[colind]))
            bound = _fast_bound(lens, absprod, y0 if beta else np.zeros(rows))
            assert np.all(np.abs(ys[0] - y_ref) <= bound)
    # the compact reduce (default) runs groups over the rows with segments only; the fill blocks give
    # the empty rows y_in (beta 1) or +0.0 (beta 0) exactly
    empty = lens == 0
    assert empty.sum() > 0 and h.stat("wcsr_rows_with_segments") == int((~empty).sum())
    ncg = h.stat("wcsr_reduce_groups")
    h.set_option("wcsr_reduce", 1)
    assert ncg <= h.stat("wcsr_reduce_groups")
    h.set_option("wcsr_reduce", 0)
    y1 = h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST)
    assert y1[empty].tobytes() == y0[empty].tobytes()
    y_zero = h.exec(x, y0.copy(), beta=0, mode=hs.MODE_FAST)
    assert np.all(y_zero[empty] == 0) and not np.signbit(y_zero[empty].astype(np.float64)).any()
    # the empty rows written after the reduce (option wcsr_fill 0) or beside the segment pass (1)
    for fill in (0, 1):
        h.set_option("wcsr_fill", fill)
        assert h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST).tobytes() == y1.tobytes()
        assert h.exec(x, y0.copy(), beta=0, mode=hs.MODE_FAST).tobytes() == y_zero.tobytes()
    h.set_option("wcsr_fill", -1)
    # the all-rows reduce (option wcsr_reduce 1): also deterministic and within the bound
    h.set_option("wcsr_reduce", 1)
    for beta in (0, 1):
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else np.zeros(rows, dtype)), rows=rows)
        ys = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(2)]
        assert ys[0].tobytes() == ys[1].tobytes()
        if dtype == np.uint64:
            assert ys[0].tobytes() == y_ref.tobytes()
        else:
            absprod = np.zeros(rows)
            np.add.at(absprod, row_of, np.abs(vals * x[colind]))
            assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(lens, absprod, y0 if beta else np.zeros(rows)))
    h.set_option("wcsr_reduce", 0)
    # the segment pass with half its groups' entries resident (option wcsr_res, k_wpass): the same bits
    y_nt = h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST)
    assert y_nt.tobytes() == y1.tobytes()
    h.set_option("wcsr_res", h.stat("wcsr_groups") // 2)
    assert h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST).tobytes() == y_nt.tobytes()
    h.set_option("wcsr_res", 0)
    if dtype == np.float64:
        with pytest.raises(hs.HipSpMVError):  # FAST only
            h.exec(x, beta=0, mode=hs.MODE_ORDERED)
    h.close()


def test_duplicates_and_cms_bits(gpu):
    # duplicate (row, col) entries are added in CSC order; CMS bits 30/31 of the
    # row ids (SparseMatrix::markRowStarts) are ignored by the backend
    colptr = np.array([0, 3, 5], np.uint32)
    rowind = np.array([0, 0, 2, 1, 1], np.uint32)
    vals = np.array([0.1, 0.2, 1e16, 3.0, -3.0], np.float64)
    x = np.array([1.7, -2.3])
    y_ref = oracle.spmv_csc(colptr, rowind, vals, x, rows=3)
    marked = rowind | np.array([1 << 31, 0, 1 << 31, 1 << 31 | 1 << 30, 1 << 30], np.uint32)
    for kernel in ORDERED_KERNELS:
        h = hs.Handle.from_csc(colptr, marked, vals, 3, 2)
        h.set_kernel(kernel)
        y = h.exec(x, beta=0)
        assert y.tobytes() == y_ref.tobytes()


def test_synthetic_c3_full_size_ordered(gpu):
    # BASELINE config C3 at full size: 2^20 x 2^20, 32 nnz/row; ordered == oracle bit for bit
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    x = hs.gen_vector(n, 3)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    h = hs.Handle.from_csc(colptr, rowind, cvals, n, n)
    assert h.kernel_name(hs.MODE_ORDERED) == "vcache"  # AUTO's ordered kernel on C3
    y = h.exec(x, beta=0, mode=hs.MODE_ORDERED)
    assert y.tobytes() == y_ref.tobytes()
    for nt in (0, 1 << 30):  # every / no row block's entries non-temporal: the same bits
        h.set_option("vcache_nt", nt)
        assert h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes()
    h.set_option("vcache_nt", -1)
    h.set_kernel("sell")
    assert h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes()
    h.set_kernel("auto")
    # the CSR entry point gives the same bits
    h2 = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h2.exec(x, beta=0).tobytes() == y_ref.tobytes()
    # fast kernel within the bound
    h.set_kernel("csr_vector")
    yf = h.exec(x, beta=0, mode=hs.MODE_FAST)
    lens = np.full(n, 32)
    absprod = np.zeros(n)
    np.add.at(absprod, np.repeat(np.arange(n), 32), np.abs(vals * x[colind]))
    assert np.all(np.abs(yf - y_ref) <= _fast_bound(lens, absprod, 0))


def test_exec_device_torch(gpu):
    import torch
    rows, cols, colptr, rowind, vals = fx.load("circuit204")
    x = np.random.default_rng(2).uniform(-1, 1, cols)
    y_ref = oracle.spmv_csc(colptr, rowind, vals, x, rows=rows)
    h = hs.Handle.from_csc(colptr, rowind, vals, rows, cols)
    h.set_option("timing", 1)
    xd = torch.from_numpy(x).to(gpu)
    yd = torch.empty(rows, dtype=torch.float64, device=gpu)
    s = torch.cuda.current_stream()
    h.exec_device(xd, yd, beta=0, mode=hs.MODE_ORDERED, stream=s)
    s.synchronize()
    assert yd.cpu().numpy().tobytes() == y_ref.tobytes()
    assert h.stat("kernel_ns") > 0
    # accumulate in place (y_in == y_out)
    h.exec_device(xd, yd, y_in=yd, beta=1, mode=hs.MODE_ORDERED, stream=s)
    s.synchronize()
    y2 = oracle.spmv_csc(colptr, rowind, vals, x, y=y_ref.copy(), rows=rows)
    assert yd.cpu().numpy().tobytes() == y2.tobytes()


def test_invalid_matrix_rejected(gpu):
    colptr = np.array([0, 2, 1], np.uint32)  # not monotone
    with pytest.raises(hs.HipSpMVError) as e:
        hs.Handle.from_csc(colptr, np.array([0, 1], np.uint32), np.ones(2), 2, 2)
    assert e.value.status == 2
    with pytest.raises(hs.HipSpMVError):
        hs.Handle.from_csc(np.array([0, 1, 2], np.uint32), np.array([0, 5], np.uint32), np.ones(2), 2, 2)


def test_plugin_surface_spmvbench(gpu):
    # software/main.cpp pipeline through HWSpMVFactory -> HIPSpMV; diffFromGolden == 0
    import subprocess
    names = fx.ALL_FIXTURES
    out = subprocess.run([f"{hs.LIB_DIR}/spmvbench", "--dir", fx.MATRICES, "--confs", "hip,hip3", "--cms", "1",
                          *names], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.splitlines()
    hdr = next(l for l in lines if l.startswith("diffFromGolden,"))
    keys = hdr.rstrip(",").split(",")
    recs = [dict(zip(keys, l.rstrip(",").split(","))) for l in lines if l[:1].isdigit()]
    assert len(recs) == 2 * len(names)
    for i, r in enumerate(recs):
        assert r["diffFromGolden"] == "0" and r["accType"] == "HIPSpMV" and r["error"] == "0", r
        assert r["numDevices"] == ("1" if i < len(names) else "3"), r
        # the GPU preprocessing statistics (SoftwareSpMV.cpp:72-95 keys), masked CMS marks
        rows, cols, colptr, rowind, _ = fx.load(r["matrix"])
        assert int(r["maxAlive"]) == oracle.max_alive(rowind, rows), r
        assert int(r["maxColSpan"]) == oracle.max_col_span(colptr, rowind), r
        # the reference NewCache keys (HardwareSpMVNewCache.cpp:189-204), restated for the GPU
        assert 0 < int(r["activeCycles"]) <= int(r["totalCycles"]), r  # roofline-time <= kernel time
        assert int(r["readMisses"]) > 0 and int(r["hazardStalls"]) >= 0, r


def _layout_runs(rowptr, colind, rows, panel):
    """entries continuing a run (same row, same panel as the previous entry): CPU count"""
    c = colind.astype(np.int64) // panel
    same = np.zeros(colind.size, bool)
    same[1:] = c[1:] == c[:-1]
    same[rowptr[:-1].astype(np.int64)[np.diff(rowptr) > 0]] = False  # a row's first entry never continues
    return int(same.sum())


def test_cache_behaviour_stats(gpu):
    """read_misses / hazard_stalls / ocm_depth / cycles per kernel, checked against the layout computed
    on the CPU: x words streamed into LDS by every row block, run continuations, y block + 2 panels"""
    n = 1 << 18
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    for kernel, mode, panel in [("vcache_split", hs.MODE_FAST, 4000), ("vcache", hs.MODE_ORDERED, 8128)]:
        h.set_kernel(kernel)
        h.exec(x, beta=0, mode=mode)
        # the layout sizes its row blocks to fill the chip (<= 12352 / 4096 rows; split: 3 column parts)
        nb = h.stat("vcache_split_units") // 3 if kernel == "vcache_split" else h.stat("vcache_blocks")
        rpb = h.stat("vcache_split_rows_per_block" if kernel == "vcache_split" else "vcache_rows_per_block")
        assert nb == -(-n // rpb)
        assert h.stat("read_misses") == nb * n, kernel  # every row block streams all of x through LDS once
        assert h.stat("hazard_stalls") == _layout_runs(rowptr, colind, n, panel), kernel
        assert h.stat("ocm_depth") == rpb + 2 * panel, kernel
        assert 0 < h.stat("active_cycles") < h.stat("total_cycles"), kernel
    for kernel, mode in [("sell", hs.MODE_ORDERED), ("csr_vector", hs.MODE_FAST)]:
        h.set_kernel(kernel)
        h.exec(x, beta=0, mode=mode)
        assert h.stat("read_misses") == colind.size, kernel  # every product gathers x from memory
        assert h.stat("hazard_stalls") == (0 if kernel == "csr_vector" else colind.size - n), kernel
        assert h.stat("ocm_depth") == 0, kernel
    h.close()


REF_NEWCACHE_KEYS = ["sActive", "sFill", "sFlush", "sDone", "sReadMiss1", "sReadMiss2", "sReadMiss3", "sColdMiss",
                     "totalCycles", "activeCycles", "readMisses", "ocmDepth", "issueWindow", "hazardStalls",
                     "capacityStalls", "cms", "noValidButReady", "noReadyButValid"]


def test_profile_state_statistics(gpu):
    """option "profile": the vcache kernels' in-kernel stamps give the NewCache cache-FSM state counts
    (HardwareSpMVNewCache.cpp:130-204) -- same bits as the unprofiled launch, and the per-workgroup
    phases (fill + active + flush + done) add up to the launch's span"""
    n = 1 << 18
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.stat("profiled") == 0 and h.stat("state_active") == 0
    for kernel, mode in [("vcache_split", hs.MODE_FAST), ("vcache", hs.MODE_ORDERED)]:
        h.set_kernel(kernel)
        y0 = h.exec(x, beta=0, mode=mode)
        h.set_option("profile", 1)
        y1 = h.exec(x, beta=0, mode=mode)
        assert y1.tobytes() == y0.tobytes(), kernel
        assert h.stat("profiled") == 1 and h.stat("profile_units") == (
            h.stat("vcache_split_units") if kernel == "vcache_split" else h.stat("vcache_blocks")), kernel
        st = {k: h.stat("state_" + k) for k in ("fill", "active", "flush", "done", "read_miss1", "read_miss2",
                                                "read_miss3", "cold_miss")}
        span = h.stat("profile_span_cycles")
        assert st["active"] > 0 and st["fill"] > 0 and st["flush"] > 0 and st["read_miss2"] > 0, (kernel, st)
        assert st["read_miss1"] == 0 and st["read_miss3"] == 0 and st["cold_miss"] == n, (kernel, st)
        phases = st["fill"] + st["active"] + st["flush"] + st["done"]
        assert 0.9 * span <= phases <= 1.01 * span, (kernel, st, span)
        # the launch's span fits inside the event-timed kernel (a few us of launch overhead around it)
        assert span <= h.stat("kernel_ns") * h.stat("clock_khz") / 1e6 * 1.05, (kernel, span)
        assert h.stat("no_valid_but_ready") + h.stat("no_ready_but_valid") > 0, kernel
        assert h.stat("issue_window") > 0 and h.stat("capacity_stalls") == 0 and h.stat("cms") == 0
        h.set_option("profile", 0)
    # a kernel without stamps leaves the last profiled launch's statistics in place
    h.set_option("profile", 1)
    h.set_kernel("sell")
    h.exec(x, beta=0, mode=hs.MODE_ORDERED)
    assert h.stat("profiled") == 1 and h.stat("issue_window") == 0
    h.close()


def test_plugin_surface_spmvbench_profile(gpu):
    """spmvbench --profile 1: the CSV carries HardwareSpMVNewCache::statKeys under the reference's names and
    order, with the state counts measured (vcache kernels)"""
    import subprocess
    names = ["circuit204", "row64k"]
    out = subprocess.run([f"{hs.LIB_DIR}/spmvbench", "--dir", fx.MATRICES, "--confs", "hip", "--cms", "0",
                          "--kernel", "vcache", "--mode", "ordered", "--profile", "1", *names],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.splitlines()
    keys = next(l for l in lines if l.startswith("diffFromGolden,")).rstrip(",").split(",")
    pos = [keys.index(k) for k in REF_NEWCACHE_KEYS]
    assert pos == sorted(pos), "NewCache keys out of the reference's order"
    recs = [dict(zip(keys, l.rstrip(",").split(","))) for l in lines if l[:1].isdigit()]
    assert len(recs) == len(names)
    for r in recs:
        assert r["diffFromGolden"] == "0" and r["error"] == "0", r
        assert int(r["sActive"]) > 0 and int(r["sFill"]) > 0 and int(r["sFlush"]) > 0, r
        assert int(r["issueWindow"]) > 0 and r["capacityStalls"] == "0" and r["cms"] == "0", r


def test_auto_fast_long_row_takes_sell(gpu):
    """AUTO FAST: a row that would outlast the rest in csr_vector (one wave per long row) goes to
    sell's hub pieces; deterministic and within the FAST bound of the oracle."""
    rng = np.random.default_rng(5)
    rows, cols = 2000, 1 << 20
    lens = np.ones(rows, np.int64)
    lens[7] = 200_000
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
    vals = rng.uniform(-1, 1, colind.size)
    x = rng.uniform(-1, 1, cols)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.kernel_name(hs.MODE_FAST) == "sell" and h.kernel_name(hs.MODE_ORDERED) == "sell"
    ys = [h.exec(x, beta=0, mode=hs.MODE_FAST) for _ in range(2)]
    assert ys[0].tobytes() == ys[1].tobytes()
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=rows)
    absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]), minlength=rows)
    assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(lens, absprod, 0))
    assert h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes()
    h.close()


def test_c3_split_deterministic_and_within_bound(gpu):
    # vcache_split: three column-part partials combined in fixed order -> identical
    # bits on every run, and within the FAST-mode bound of the oracle
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.stat("vcache_split_eligible") == 1
    assert h.kernel_name(hs.MODE_FAST) == "vcache_split"
    # x streamed into LDS per launch: 256 ordered units x 8 MB; 85 split row blocks x 8 MB (3 parts x 1/3 each)
    assert h.stat("vcache_x_bytes") == 256 * 8 * n and h.stat("vcache_split_x_bytes") == 85 * 8 * n
    assert h.stat("vcache_split_units") == 255 and h.stat("vcache_split_rows_per_block") == -(-n // 85)
    ys = [h.exec(x, beta=0, mode=hs.MODE_FAST) for _ in range(3)]
    assert ys[0].tobytes() == ys[1].tobytes() == ys[2].tobytes()
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    absprod = np.zeros(n)
    np.add.at(absprod, np.repeat(np.arange(n), 32), np.abs(vals * x[colind]))
    assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(np.full(n, 32), absprod, 0))
    # beta = 1 accumulates y_in into part 0 only
    y0 = np.random.default_rng(4).uniform(-1, 1, n)
    y1 = h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST)
    assert np.all(np.abs(y1 - (y_ref + y0)) <= _fast_bound(np.full(n, 33), absprod + np.abs(y0), 0) * 2)


@pytest.mark.parametrize("vmap", [0, 1])
def test_vflow_c3_full_size(gpu, vmap):
    if not hs.experimental_build():
        pytest.skip("k_vflow: experimental build only (HIPSPMV_EXPERIMENTAL=1)")
    # k_vflow (csrc/vflow.hip) on full C3: 64 row blocks x 4 parts = 256 units, x streamed into LDS
    # 64 x 8 MB per launch; deterministic (identical bits on every launch and under either XCD
    # placement), within the FAST bound of the oracle, u64 exact, no flag wait gave up
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("vcache_flow")
    h.set_option("vflow_map", vmap)
    assert h.stat("vflow_eligible") == 1 and h.stat("vflow_units") == 256
    assert h.stat("vflow_x_bytes") == 64 * 8 * n and h.stat("vflow_max_group") <= 128
    ys = [h.exec(x, beta=0, mode=hs.MODE_FAST) for _ in range(3)]
    assert ys[0].tobytes() == ys[1].tobytes() == ys[2].tobytes()
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    absprod = np.zeros(n)
    np.add.at(absprod, np.repeat(np.arange(n), 32), np.abs(vals * x[colind]))
    assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(np.full(n, 32), absprod, 0))
    y0 = np.random.default_rng(4).uniform(-1, 1, n)
    y1 = h.exec(x, y0.copy(), beta=1, mode=hs.MODE_FAST)
    assert np.all(np.abs(y1 - (y_ref + y0)) <= _fast_bound(np.full(n, 33), absprod + np.abs(y0), 0) * 2)
    assert h.stat("vflow_timeouts") == 0
    h.close()
    uv = (vals.view(np.uint64) >> np.uint64(7))
    ux = np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    hu = hs.Handle.from_csr(rowptr, colind, uv, n, n)
    hu.set_kernel("vcache_flow")
    hu.set_option("vflow_map", vmap)
    _, _, cuv = oracle.csr2csc(n, n, rowptr, colind, uv)
    assert hu.exec(ux, beta=0, mode=hs.MODE_FAST).tobytes() == oracle.spmv_csc(colptr, rowind, cuv, ux, rows=n).tobytes()
    assert hu.stat("vflow_timeouts") == 0
    hu.close()


def test_split_combine_concurrent_streams(gpu):
    # vcache_split's column-part combine uses per-handle tickets and partials;
    # launches of one handle on two streams with no host synchronisation are
    # ordered by the handle (include/hipspmv.h), so every result is the
    # single-stream one, bit for bit
    import torch
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.kernel_name(hs.MODE_FAST) == "vcache_split"
    xs = [torch.from_numpy(hs.gen_vector(n, 3 + i)).cuda() for i in range(2)]
    want = []
    for x in xs:
        y = torch.empty(n, dtype=torch.float64, device="cuda")
        h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        want.append(y.cpu().numpy().tobytes())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(8)] for _ in range(2)]
    torch.cuda.synchronize()
    for k in range(8):
        for i in range(2):
            h.exec_device(xs[i], outs[i][k], beta=0, mode=hs.MODE_FAST, stream=streams[i])
    # and the host-buffer path (the handle's own stream) in between
    y_host = h.exec(xs[0].cpu().numpy(), beta=0, mode=hs.MODE_FAST)
    torch.cuda.synchronize()
    assert y_host.tobytes() == want[0]
    for i in range(2):
        for k in range(8):
            assert outs[i][k].cpu().numpy().tobytes() == want[i], (i, k)


# ---- k_vquad (vcache_split4, csrc/vquad.hip): four column parts, x panels in
# flight in registers; every configuration on the full C3 matrix and on
# ragged / wide shapes: deterministic, within the FAST bound, u64 exact; the
# forced combine fallback (variant 20) counted
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26])
def test_vquad_variants(gpu, variant):  # configurations: x / entry ring depths (csrc/vquad.hip)
    if not hs.experimental_build():
        pytest.skip("k_vquad: experimental build only (HIPSPMV_EXPERIMENTAL=1)")
    cases = [(1 << 20, 1 << 20), (70001, 13001), (3000, 20001), (65536, 1 << 20), (20000, 1 << 22),
             (16385, 7937)]
    ran = 0
    for rows, cols in cases:
        rng = np.random.default_rng(rows + variant)
        if cols >= 1 << 20:
            rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
        else:
            lens = rng.integers(0, 12, rows)
            rowptr = np.zeros(rows + 1, np.uint32)
            rowptr[1:] = np.cumsum(lens)
            colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
            vals = rng.uniform(-1, 1, colind.size)
        x = rng.uniform(-1, 1, cols)
        h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
        try:  # the stat is the shape's eligibility; the lane placement decides on selection
            if not h.stat("vcache_split4_eligible"):
                raise hs.HipSpMVError(5, "not eligible")
            h.set_kernel("vcache_split4")
        except hs.HipSpMVError:
            h.close()
            continue
        h.set_option("vquad_variant", variant)
        if variant in (22, 23, 25):  # row block 0 resident (default policy), the others non-temporal
            h.set_option("vcache_nt", 1)
        colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        lens = np.diff(rowptr.astype(np.int64))
        absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]), minlength=rows)
        for beta in (0, 1):
            y0 = rng.uniform(-1, 1, rows)
            y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
            ys = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(2)]
            assert ys[0].tobytes() == ys[1].tobytes(), (rows, cols, beta)  # deterministic
            bound = 2.0 * (lens + 1) * 2.0 ** -53 * (absprod + (np.abs(y0) if beta else 0)) + 1e-300
            assert np.all(np.abs(ys[0] - y_ref) <= bound), (rows, cols, beta)
        if rows <= 70001:  # the u64 semiring: exact mod 2^64
            uv = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
            ux = rng.integers(0, 2**64, cols, dtype=np.uint64)
            hu = hs.Handle.from_csr(rowptr, colind, uv, rows, cols)
            hu.set_kernel("vcache_split4")
            hu.set_option("vquad_variant", variant)
            if variant in (22, 23, 25):
                hu.set_option("vcache_nt", 1)
            _, _, cuv = oracle.csr2csc(rows, cols, rowptr, colind, uv)
            assert hu.exec(ux, beta=0, mode=hs.MODE_FAST).tobytes() == \
                oracle.spmv_csc(colptr, rowind, cuv, ux, rows=rows).tobytes(), (rows, cols)
            if variant == 20:  # every owner gave up: the publish-and-count path ran (and was exact)
                assert hu.stat("handoff_fallbacks") > 0
            hu.close()
        if variant == 20:
            assert h.stat("handoff_fallbacks") > 0
        h.close()
        ran += 1
    assert ran >= 3  # shapes whose runs the lane placement cannot keep inside waves are not eligible


@pytest.mark.parametrize("xlane", [3, 4])
def test_vcache_split_entry_loads(gpu, xlane):  # 3: clamped entry loads; 4: masked past the segment
    if xlane == 4 and not hs.experimental_build():
        pytest.skip("vcache_xlane 4: experimental build only (HIPSPMV_EXPERIMENTAL=1)")
    cases = [(1 << 20, 1 << 20), (70001, 13001), (3000, 20001), (65536, 1 << 20), (16385, 12001)]
    ran = 0
    for rows, cols in cases:
        rng = np.random.default_rng(rows + 7 * xlane)
        if cols >= 1 << 20:
            rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
        else:
            lens = rng.integers(0, 14, rows)
            rowptr = np.zeros(rows + 1, np.uint32)
            rowptr[1:] = np.cumsum(lens)
            colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
            vals = rng.uniform(-1, 1, colind.size)
        x = rng.uniform(-1, 1, cols)
        h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
        if not h.stat("vcache_split_eligible"):
            h.close()
            continue
        h.set_kernel("vcache_split")
        h.set_option("vcache_xlane", xlane)
        colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        lens = np.diff(rowptr.astype(np.int64))
        absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]), minlength=rows)
        for beta in (0, 1):
            y0 = rng.uniform(-1, 1, rows)
            y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
            ys = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(2)]
            assert ys[0].tobytes() == ys[1].tobytes(), (rows, cols, beta)  # deterministic
            bound = 2.0 * (lens + 1) * 2.0 ** -53 * (absprod + (np.abs(y0) if beta else 0)) + 1e-300
            assert np.all(np.abs(ys[0] - y_ref) <= bound), (rows, cols, beta)
        if rows <= 70001:  # the u64 semiring: exact mod 2^64
            uv = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
            ux = rng.integers(0, 2**64, cols, dtype=np.uint64)
            hu = hs.Handle.from_csr(rowptr, colind, uv, rows, cols)
            hu.set_kernel("vcache_split")
            hu.set_option("vcache_xlane", xlane)
            _, _, cuv = oracle.csr2csc(rows, cols, rowptr, colind, uv)
            assert hu.exec(ux, beta=0, mode=hs.MODE_FAST).tobytes() == \
                oracle.spmv_csc(colptr, rowind, cuv, ux, rows=rows).tobytes(), (rows, cols)
            hu.close()
        h.close()
        ran += 1
    assert ran >= 3


@pytest.mark.parametrize("xlane,xmask", [(-1, 1), (0, 1), (6, 1), (6, 0), (0, 0)])
def test_ordered_vcache_continuation_and_xmask(gpu, xlane, xmask):
    # the ORDERED vcache's run continuations (6, the default on banked layouts: the first continuation
    # entry from the next lane by DPP, the rest re-read from memory; 0: all re-read) and its x-line mask
    # (loaders skip the x lines no entry of a panel uses): bit-exact to SoftwareSpMV, f64 and u64, on
    # rows with runs of one, two and many entries per panel (dense rows: runs up to hundreds long)
    cases = [(65536, 1 << 20, None), (5000, 20001, 0.002), (257, 12161, 0.3), (70000, 13001, 0.0008)]
    for rows, cols, dens in cases:
        rng = np.random.default_rng(rows + cols)
        if dens is None:
            rowptr, colind, vals = hs.gen_stripe_csr(3, rows, cols, 32)
        else:
            lens = rng.binomial(cols, dens, rows)
            rowptr = np.zeros(rows + 1, np.uint32)
            rowptr[1:] = np.cumsum(lens)
            colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
            vals = rng.uniform(-1, 1, colind.size)
        x = rng.uniform(-1, 1, cols)
        h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
        if not h.stat("vcache_eligible"):
            h.close()
            continue
        h.set_kernel("vcache")
        h.set_option("vcache_xlane", xlane)
        h.set_option("vcache_xmask", xmask)
        colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        for beta in (0, 1):
            y0 = rng.uniform(-1, 1, rows)
            y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
            assert h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes(), \
                (rows, cols, beta)
        uv = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
        ux = rng.integers(0, 2**64, cols, dtype=np.uint64)
        hu = hs.Handle.from_csr(rowptr, colind, uv, rows, cols)
        hu.set_kernel("vcache")
        hu.set_option("vcache_xlane", xlane)
        hu.set_option("vcache_xmask", xmask)
        _, _, cuv = oracle.csr2csc(rows, cols, rowptr, colind, uv)
        assert hu.exec(ux, beta=0, mode=hs.MODE_ORDERED).tobytes() == \
            oracle.spmv_csc(colptr, rowind, cuv, ux, rows=rows).tobytes(), (rows, cols)
        hu.close()
        h.close()


def test_vquad_c3_full_size(gpu):
    if not hs.experimental_build():
        pytest.skip("k_vquad: experimental build only (HIPSPMV_EXPERIMENTAL=1)")
    # the four-part kernel on full C3: x streamed into LDS per launch is 64 row
    # blocks x 8 MB (three parts: 85 x 8 MB); deterministic and within the bound
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.stat("vcache_split4_eligible") == 1
    h.set_kernel("vcache_split4")
    assert h.stat("vcache_split4_x_bytes") == 64 * 8 * n
    ys = [h.exec(x, beta=0, mode=hs.MODE_FAST) for _ in range(3)]
    assert ys[0].tobytes() == ys[1].tobytes() == ys[2].tobytes()
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    absprod = np.zeros(n)
    np.add.at(absprod, np.repeat(np.arange(n), 32), np.abs(vals * x[colind]))
    assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(np.full(n, 32), absprod, 0))
    assert h.stat("handoff_fallbacks") >= 0  # readable; the owner waits normally succeed (co-resident parts)


# ---- experimental vcache variants (never chosen by AUTO): four column parts
# and the LDS-DMA x loader.  Addressing is replayed on the CPU by
# tests/test_vcache_sim.py; on the GPU they run only with HIPSPMV_EXPERIMENTAL=1
# until they have been measured on an MI355X.
EXPERIMENTAL = os.environ.get("HIPSPMV_EXPERIMENTAL") == "1"  # (the library is then lib/exp's)


@pytest.mark.skipif(not EXPERIMENTAL, reason="experimental kernels: set HIPSPMV_EXPERIMENTAL=1")
@pytest.mark.parametrize("kernel,dma,xlane,xmap", [
    ("vcache_split", 1, 0, 0), ("vcache", 1, 0, 0),
    ("wgather", 0, 0, 0), ("vcache", 0, 1, 0), ("vcache", 0, 2, 0), ("vcache_split", 0, 1, 0),
    ("vcache_split", 0, 2, 0), ("vcache_split", 1, 2, 0), ("wgather", 0, 2, 0),
    ("vcache", 0, 3, 0), ("vcache_split", 0, 3, 0)])
def test_experimental_vcache_variants(gpu, kernel, dma, xlane, xmap):
    cases = [(1 << 20, 1 << 20), (70001, 13001), (3000, 20001), (65536, 1 << 20), (20000, 1 << 22)]
    for rows, cols in cases:
        rng = np.random.default_rng(rows)
        if cols >= 1 << 20:
            rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
        else:
            lens = rng.integers(0, 12, rows)
            rowptr = np.zeros(rows + 1, np.uint32)
            rowptr[1:] = np.cumsum(lens)
            colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
            vals = rng.uniform(-1, 1, colind.size)
        x = rng.uniform(-1, 1, cols)
        h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
        key = {"vcache_split4": "vcache_split4_eligible", "vcache_split": "vcache_split_eligible",
               "wgather": "wgather_eligible"}.get(kernel, "vcache_eligible")
        if not h.stat(key):
            continue
        try:
            h.set_kernel(kernel)
        except hs.HipSpMVError:  # a four-part layout not placeable for this shape
            continue
        h.set_option("vcache_dma", dma)
        h.set_option("vcache_xlane", xlane)
        h.set_option("vcache_map", xmap)
        mode = hs.MODE_ORDERED if kernel in ("vcache", "wgather") else hs.MODE_FAST
        colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        for beta in (0, 1):
            y0 = rng.uniform(-1, 1, rows)
            y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
            ys = [h.exec(x, y0.copy(), beta=beta, mode=mode) for _ in range(2)]
            assert ys[0].tobytes() == ys[1].tobytes()  # deterministic
            if mode == hs.MODE_ORDERED:
                assert ys[0].tobytes() == y_ref.tobytes(), (rows, cols, beta)
            else:
                lens = np.diff(rowptr.astype(np.int64))
                absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]),
                                      minlength=rows)
                bound = 2.0 * (lens + 1) * 2.0 ** -53 * (absprod + (np.abs(y0) if beta else 0)) + 1e-300
                assert np.all(np.abs(ys[0] - y_ref) <= bound), (rows, cols, beta)
        h.close()


# ---- analogues of the backend known-answer test (chisel/tests/TestSpMVBackend.scala:122-178):
# write-out mode (rows come back unchanged: y_in -> y_out with nothing to add) and the stream
# sums sumUpTo(64) = 2080 carried by the nonzero-value stream and by the input-vector stream.
@pytest.mark.parametrize("kernel", ["auto", "vcache", "csr_lane", "csr_vector", "vcache_split", "sell"])
def test_backend_kat_writeout_empty_matrix(gpu, kernel):
    rows = cols = 64
    colptr = np.zeros(cols + 1, np.uint32)
    h = hs.Handle.from_csc(colptr, np.zeros(0, np.uint32), np.zeros(0, np.uint64), rows, cols)
    if kernel != "auto":
        try:
            h.set_kernel(kernel)
            h.exec(np.ones(cols, np.uint64), np.zeros(rows, np.uint64), beta=1, mode=hs.MODE_FAST)
        except hs.HipSpMVError:
            pytest.skip(f"{kernel} not applicable to an empty matrix")
    y_in = np.arange(rows, dtype=np.uint64)
    for mode in (hs.MODE_ORDERED, hs.MODE_FAST):
        try:
            y = h.exec(np.ones(cols, np.uint64), y_in.copy(), beta=1, mode=mode)
        except hs.HipSpMVError:
            continue  # a FAST-only kernel in ORDERED mode
        assert np.array_equal(y, np.arange(rows, dtype=np.uint64))
        y0 = h.exec(np.ones(cols, np.uint64), y_in.copy(), beta=0, mode=mode)
        assert not y0.any()


@pytest.mark.parametrize("kernel", ["auto", "vcache", "csr_lane", "csr_vector", "vcache_split", "sell"])
def test_backend_kat_stream_sums(gpu, kernel):
    n = 64
    # value stream i+1 in one row, x = 1: y0 = sumUpTo(64)
    colptr = np.arange(n + 1, dtype=np.uint32)
    rowvec = hs.Handle.from_csc(colptr, np.zeros(n, np.uint32), np.arange(1, n + 1, dtype=np.uint64), 1, n)
    # input-vector stream i+1 through the identity: sum(y) = sumUpTo(64)
    ident = hs.Handle.from_csc(colptr, np.arange(n, dtype=np.uint32), np.ones(n, np.uint64), n, n)
    for h, x, check in ((rowvec, np.ones(n, np.uint64), lambda y: int(y[0]) == 2080),
                        (ident, np.arange(1, n + 1, dtype=np.uint64), lambda y: int(y.sum()) == 2080)):
        if kernel != "auto":
            try:
                h.set_kernel(kernel)
                h.exec(x, beta=0, mode=hs.MODE_FAST)
            except hs.HipSpMVError:
                continue
        assert check(h.exec(x, beta=0, mode=hs.MODE_FAST)), kernel


def test_integration_example_program(gpu):
    # INTEGRATION.md section A, compiled (tools/plugin_example.cpp): factory ->
    # HIPSpMV on one device and on three blocks of this process, memcmp golden
    import subprocess
    out = subprocess.run([f"{hs.LIB_DIR}/plugin_example", fx.MATRICES, "circuit204", "3"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [l for l in out.stdout.splitlines() if l.startswith("HIPSpMV")]
    assert len(lines) == 2 and all("diffFromGolden=0" in l for l in lines), out.stdout
    assert "devices=1" in lines[0] and "devices=3" in lines[1]


# ---- k_sell (csrc/sell.hip): SELL-C-sigma lane per row, hub rows one wave each.
# Its layout and index arithmetic are replayed on the CPU by tests/test_sell_sim.py.
def test_sell_rmat_hubs_ordered_and_fast(gpu):
    rowptr, colind, vals = hs.gen_rmat_csr(15)
    n = 1 << 15
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("sell")
    assert h.kernel_name(hs.MODE_ORDERED) == "sell" and h.stat("sell_hubs") > 0
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    x = hs.gen_vector(n, 3)
    lens = np.diff(rowptr.astype(np.int64))
    absprod = np.bincount(np.repeat(np.arange(n), lens), weights=np.abs(vals * x[colind]), minlength=n)
    for beta in (0, 1):
        y0 = np.random.default_rng(beta).uniform(-1, 1, n)
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=n)
        y = h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_ORDERED)
        assert y.tobytes() == y_ref.tobytes(), beta
        yf = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(2)]
        assert yf[0].tobytes() == yf[1].tobytes()  # deterministic
        bound = _fast_bound(lens + 1, absprod, y0 if beta else np.zeros(n))
        assert np.all(np.abs(yf[0] - y_ref) <= bound), beta
    h.close()


def test_sell_c3_full_size_ordered(gpu):
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    x = hs.gen_vector(n, 3)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("sell")
    assert h.stat("sell_padding") == 0 and h.stat("sell_hubs") == 0
    assert h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes()
    h.close()


def test_plugin_surface_spmvbench_sell(gpu):
    # the plugin pipeline with the SELL kernel register, one device and three
    import subprocess
    names = fx.ALL_FIXTURES
    out = subprocess.run([f"{hs.LIB_DIR}/spmvbench", "--dir", fx.MATRICES, "--confs", "hip,hip3", "--cms", "1",
                          "--kernel", "sell", *names], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.splitlines()
    hdr = next(l for l in lines if l.startswith("diffFromGolden,"))
    keys = hdr.rstrip(",").split(",")
    recs = [dict(zip(keys, l.rstrip(",").split(","))) for l in lines if l[:1].isdigit()]
    assert len(recs) == 2 * len(names)
    for r in recs:
        assert r["diffFromGolden"] == "0" and r["error"] == "0" and r["kernel"] == "7", r


def test_sell_split_hub_rows_fast(gpu):
    # FAST hub rows over 4096 entries are cut into pieces whose partials the
    # last-finishing piece adds in piece order; tickets reset themselves, so
    # repeated launches must give identical bits
    rng = np.random.default_rng(21)
    rows, cols = 700, 30000
    lens = np.full(rows, 3)
    lens[[0, 333, 699]] = [20000, 4097, 8192]
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
    vals = rng.uniform(-1, 1, colind.size)
    x = rng.uniform(-1, 1, cols)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    h.set_kernel("sell")
    assert h.stat("sell_hubs") == 3 and h.stat("sell_hub_pieces") == 9
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]), minlength=rows)
    for beta in (0, 1):
        y0 = rng.uniform(-1, 1, rows)
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
        ys = [h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST) for _ in range(3)]
        assert ys[0].tobytes() == ys[1].tobytes() == ys[2].tobytes()
        assert np.all(np.abs(ys[0] - y_ref) <= _fast_bound(lens + 1, absprod, y0 if beta else np.zeros(rows)))
        assert h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_ORDERED).tobytes() == y_ref.tobytes()
    # u64: pieces and combine are exact mod 2^64
    vu = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
    xu = rng.integers(0, 2**64, cols, dtype=np.uint64)
    hu = hs.Handle.from_csr(rowptr, colind, vu, rows, cols)
    hu.set_kernel("sell")
    cp, ri, cv = oracle.csr2csc(rows, cols, rowptr, colind, vu)
    want = oracle.spmv_csc(cp, ri, cv, xu, rows=rows)
    for _ in range(2):
        assert hu.exec(xu, beta=0, mode=hs.MODE_FAST).tobytes() == want.tobytes()
    h.close()
    hu.close()


def test_sell_isolated_hub_chains_ordered(gpu):
    # ORDERED hub rows of >= 8192 entries (kSellIso) run as isolated chains,
    # one 1024-thread workgroup each, fed from LDS by helper waves
    # (hub_row_isolated): the oracle's bits at stage-boundary lengths (the
    # stages hold 64*G products), just below the threshold, and beside empty
    # rows and short-row slices
    rng = np.random.default_rng(29)
    rows, cols = 900, 120000
    lens = rng.integers(0, 40, rows)
    lens[[0, 5, 6, 7, 400, 899]] = [100001, 8191, 8192, 8193, 30720, 20481]
    lens[[1, 2]] = 0
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate([np.sort(rng.choice(cols, n, replace=False)) for n in lens]).astype(np.uint32)
    vals = rng.uniform(-1, 1, colind.size)
    x = rng.uniform(-1, 1, cols)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    h.set_kernel("sell")
    assert h.stat("sell_iso_hubs") == 5
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    for beta in (0, 1):
        y0 = rng.uniform(-1, 1, rows)
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
        for _ in range(2):
            y = h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_ORDERED)
            bad = np.nonzero(y.view(np.uint64) != y_ref.view(np.uint64))[0]
            assert bad.size == 0, (beta, bad[:8], lens[bad[:8]])
    h.close()


def test_exec_device_rejects_bad_tensors(gpu):
    import torch
    rows, cols, colptr, rowind, vals = fx.load("circuit204")
    h = hs.Handle.from_csc(colptr, rowind, vals, rows, cols)
    x = torch.zeros(cols, dtype=torch.float64, device=gpu)
    y = torch.empty(rows, dtype=torch.float64, device=gpu)
    for bad_x, bad_y in ((x[:-1], y), (x, y[:-1]), (x, torch.empty(2 * rows, dtype=torch.float64, device=gpu)[::2]),
                         (x.cpu(), y), (x.float(), y)):
        with pytest.raises(ValueError):
            h.exec_device(bad_x, bad_y, beta=0, mode=hs.MODE_ORDERED)
    h.close()


def test_split_eligible_at_four_panels(gpu):
    # 12001-16000 columns give the split geometry 4 panels: parts of 1, 1, 2 (a ceil cut left the
    # third part empty and the matrix ineligible)
    rng = np.random.default_rng(3)
    colptr, rowind, vals = _random_csc(1500, 14001, 0.003, rng)
    h = hs.Handle.from_csc(colptr, rowind, vals, 1500, 14001)
    assert h.stat("vcache_split_eligible") == 1
    x = rng.uniform(-1, 1, 14001)
    for beta in (0, 1):
        _check("4 panels", 1500, 14001, colptr, rowind, vals, x, "vcache_split", beta, hs.MODE_FAST)


@pytest.mark.parametrize("kernel", ["vcache_split", "wgather_split"])
def test_graph_capture_after_eager_launch_on_another_stream(gpu, kernel):
    # A scratch kernel (tickets + partials) launched eagerly on stream A, then captured
    # on a fresh stream B: the library neither waits on nor records its scratch event inside the
    # capture, the replays give the eager bits, and eager launches on A resume after it.
    import torch
    n, cols = (1 << 16, 1 << 16) if kernel == "vcache_split" else (1 << 15, (1 << 21) + 7)
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, cols, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, cols)
    h.set_kernel(kernel)
    xd = torch.from_numpy(hs.gen_vector(cols, 3)).cuda()
    ya, yb = (torch.empty(n, dtype=torch.float64, device="cuda") for _ in range(2))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    h.exec_device(xd, ya, beta=0, mode=hs.MODE_FAST, stream=sa)
    torch.cuda.synchronize()
    ref = ya.cpu().numpy().copy()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sb):
        for _ in range(3):
            h.exec_device(xd, yb, beta=0, mode=hs.MODE_FAST, stream=sb)
    with torch.cuda.stream(sb):
        g.replay()
        g.replay()
    torch.cuda.synchronize()
    assert yb.cpu().numpy().tobytes() == ref.tobytes()
    h.exec_device(xd, ya, beta=0, mode=hs.MODE_FAST, stream=sa)
    torch.cuda.synchronize()
    assert ya.cpu().numpy().tobytes() == ref.tobytes()


def test_auto_layouts_built_at_create(gpu):
    # AUTO's layouts (here ORDERED -> vcache, FAST -> vcache_split) exist after create and count as
    # setup; a kernel selected by name builds its layout then, timed in layout_ns and setup_ns
    n = 1 << 16
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.kernel_name(hs.MODE_ORDERED) == "vcache" and h.kernel_name(hs.MODE_FAST) == "vcache_split"
    assert h.stat("sell_slices") == 0 and h.stat("auto_fallback") == 0
    x = hs.gen_vector(n, 3)
    y_o = h.exec(x, beta=0, mode=hs.MODE_ORDERED)
    h.exec(x, beta=0, mode=hs.MODE_FAST)
    assert h.stat("layout_ns") == 0 and h.stat("setup_ns") == h.stat("create_ns") > 0
    phases = sum(h.stat(f"setup_{k}_ns") for k in ("csr", "upload", "scan", "layouts"))
    assert 0 < phases <= h.stat("create_ns")  # create's phases lie inside it
    h.set_kernel("sell")  # the SELL layout: built now, from the device CSR copy
    assert h.stat("layout_ns") > 0 and h.stat("setup_ns") == h.stat("create_ns") + h.stat("layout_ns")
    assert h.stat("sell_slices") > 0
    assert h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes() == y_o.tobytes()


def test_wgather_chunked_launches_bit_identical(gpu):
    # k_wgather runs its row blocks in launches of `wgather_chunk` (kWgChunk = 256: one per CU);
    # any chunking gives the single-launch bits, ORDERED == the oracle
    rows, cols = 1 << 17, 1 << 21  # 8 row blocks of 16384
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.kernel_name(hs.MODE_ORDERED) == "wgather" and h.stat("wgather_chunk") == 256
    x = hs.gen_vector(cols, 3)
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=rows)
    outs = []
    for chunk in (0, 256, 3, 1):
        h.set_option("wgather_chunk", chunk)
        outs.append(h.exec(x, beta=0, mode=hs.MODE_ORDERED).tobytes())
    assert all(o == y_ref.tobytes() for o in outs)


@pytest.mark.parametrize("dtype", [np.float64, np.uint64])
def test_wgather_runs_and_line_order(gpu, dtype):
    # the wgather layout sorts each segment's row runs by x line: rows with several entries in
    # one 2^16-column window (runs), empty rows, a ragged last block -- ORDERED bit-exact vs
    # the oracle for beta 0 and 1, u64 exact
    rng = np.random.default_rng(5)
    rows, cols = 40001, (1 << 21) + 5
    per_row = []
    for r in range(rows):
        n = int(rng.integers(0, 12))
        w = rng.integers(0, cols >> 16, 3)  # entries clustered in up to three windows
        c = (w[rng.integers(0, 3, n)] << 16) + rng.integers(0, 1 << 16, n)
        per_row.append(np.unique(np.minimum(c, cols - 1)))
    lens = np.array([c.size for c in per_row], np.int64)
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate(per_row).astype(np.uint32)
    if dtype == np.float64:
        vals, x = rng.uniform(-1, 1, colind.size), rng.uniform(-1, 1, cols)
        y0 = rng.uniform(-1, 1, rows)
    else:
        vals = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
        x = rng.integers(0, 2**64, cols, dtype=np.uint64)
        y0 = rng.integers(0, 2**64, rows, dtype=np.uint64)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.stat("wgather_eligible")
    h.set_kernel("wgather")
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    for beta in (0, 1):
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
        y = h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_ORDERED)
        assert y.tobytes() == y_ref.tobytes(), (dtype, beta)
    h.close()


def _clustered_wide(rng, rows, cols, dtype):
    per_row = []
    for r in range(rows):
        n = int(rng.integers(0, 12))
        w = rng.integers(0, cols >> 16, 3)  # entries clustered in up to three windows
        c = (w[rng.integers(0, 3, n)] << 16) + rng.integers(0, 1 << 16, n)
        per_row.append(np.unique(np.minimum(c, cols - 1)))
    lens = np.array([c.size for c in per_row], np.int64)
    rowptr = np.zeros(rows + 1, np.uint32)
    rowptr[1:] = np.cumsum(lens)
    colind = np.concatenate(per_row).astype(np.uint32)
    if dtype == np.float64:
        return rowptr, colind, rng.uniform(-1, 1, colind.size), rng.uniform(-1, 1, cols), rng.uniform(-1, 1, rows)
    return (rowptr, colind, rng.integers(0, 2**64, colind.size, dtype=np.uint64),
            rng.integers(0, 2**64, cols, dtype=np.uint64), rng.integers(0, 2**64, rows, dtype=np.uint64))


@pytest.mark.parametrize("dtype", [np.float64, np.uint64])
@pytest.mark.parametrize("shape", ["stripe", "clustered", "ragged"])
def test_wgather_split_fast(gpu, dtype, shape):
    # k_wgather_split (two column halves, y = p0 + p1, part 0 on XCDs 0-3): AUTO's FAST kernel for
    # wide x with <= 2^21 rows; ORDERED stays on wgather.  Within the FAST bound of the oracle's
    # sums at beta 0 / 1, deterministic, u64 exact; any launch chunking (2 units per block, an odd
    # grid tail of fewer than 8 units) gives the same bits
    rng = np.random.default_rng(11)
    if shape == "stripe":
        rows, cols = 1 << 17, 1 << 21
        rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
        x, y0 = rng.uniform(-1, 1, cols), rng.uniform(-1, 1, rows)
        if dtype == np.uint64:
            vals = rng.integers(0, 2**64, colind.size, dtype=np.uint64)
            x, y0 = rng.integers(0, 2**64, cols, dtype=np.uint64), rng.integers(0, 2**64, rows, dtype=np.uint64)
    else:
        rows, cols = (40001, (1 << 21) + 5) if shape == "clustered" else (300, (1 << 21) + 3)
        rowptr, colind, vals, x, y0 = _clustered_wide(rng, rows, cols, dtype)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.stat("wgather_split_eligible")
    assert h.kernel_name(hs.MODE_FAST) == "wgather_split"
    assert h.kernel_name(hs.MODE_ORDERED) == ("wgather" if dtype == np.float64 else "wgather_split")
    assert h.stat("wgather_split_units") == 2 * -(-rows // h.stat("wgather_split_rows_per_block"))
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    lens = np.diff(rowptr.astype(np.int64))
    for beta in (0, 1):
        y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, y=(y0.copy() if beta else None), rows=rows)
        outs = []
        for chunk in (256, 256, 0, 3, 1):
            h.set_option("wgather_chunk", chunk)
            outs.append(h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST))
        h.set_option("wgather_chunk", 256)
        # entry residency (option vcache_nt: the first non-temporal block; -1 the budget rule): a cache
        # policy, the same bits
        for nt in (0, 1, 1 << 20, -1):
            h.set_option("vcache_nt", nt)
            outs.append(h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST))
        h.set_option("wgather_map", 1)  # the halves alternating over the XCDs (A/B placement): same bits
        outs.append(h.exec(x, y0.copy(), beta=beta, mode=hs.MODE_FAST))
        h.set_option("wgather_map", 0)
        assert all(o.tobytes() == outs[0].tobytes() for o in outs), (shape, beta)
        y = outs[0]
        if dtype == np.uint64:
            assert y.tobytes() == y_ref.tobytes(), (shape, beta)
        else:
            absprod = np.bincount(np.repeat(np.arange(rows), lens), weights=np.abs(vals * x[colind]), minlength=rows)
            bound = 2.0 * (lens + 1) * 2.0 ** -53 * (absprod + (np.abs(y0) if beta else 0)) + 1e-300
            assert np.all(np.abs(y - y_ref) <= bound), (shape, beta)
    h.close()


def test_stream_bandwidth(gpu):
    # the bench's second denominator (hipspmv_stream_bandwidth, csrc/stream.hip): plausible GB/s on an MI355X
    cp, rd = hs.stream_bandwidth(0, 1 << 28, 5)
    assert 1000 < cp < 8000 and 1000 < rd < 8000, (cp, rd)


def test_live_cache_statistics_from_rocprofv3(gpu, tmp_path):
    """The reference reads its cache counters from the accelerator after every
    run (HardwareSpMVNewCache.cpp:161-173).  Here: spmvbench runs once as a
    fresh child under `rocprofv3 --pmc TCC_MISS SQ_LDS_BANK_CONFLICT` (the
    program right after --), then again with that run's counter CSV (--pmc):
    the row's readMisses / hazardStalls equal the profiled run's counters of
    the kernel that ran, matched by its name."""
    import csv
    import glob
    import shutil
    import subprocess
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    bench = [f"{hs.LIB_DIR}/spmvbench", "--dir", fx.MATRICES, "--confs", "hip", "--cms", "0", "--mode", "fast",
             "--reps", "5", "circuit204"]
    out_dir = tmp_path / "pmc"
    prof = subprocess.run([exe, "--pmc", "TCC_MISS", "SQ_LDS_BANK_CONFLICT", "-d", str(out_dir), "-o", "run",
                           "--output-format", "csv", "--"] + bench, capture_output=True, text=True, timeout=120,
                          env=dict(os.environ, TMPDIR="/tmp"))
    assert prof.returncode == 0, prof.stdout[-2000:] + prof.stderr[-2000:]
    csvs = glob.glob(str(out_dir / "**" / "*counter_collection.csv"), recursive=True)
    assert csvs, prof.stdout[-2000:]
    run = subprocess.run(bench[:-1] + ["--pmc", csvs[0], "circuit204"], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stdout + run.stderr
    lines = run.stdout.splitlines()
    keys = next(l for l in lines if l.startswith("diffFromGolden,")).rstrip(",").split(",")
    rec = dict(zip(keys, [l for l in lines if l[:1].isdigit()][-1].rstrip(",").split(",")))
    # the kernel that ran: the hipspmv kernel of the profiled run (one SpMV per spmvbench row)
    per = {}
    with open(csvs[0]) as f:
        for row in csv.DictReader(f):
            if "hipspmv::" in row["Kernel_Name"]:
                per.setdefault((row["Kernel_Name"], row["Counter_Name"]), {})[row["Dispatch_Id"]] = \
                    float(row["Counter_Value"])
    names = {k for k, _ in per}
    main = max(names, key=lambda n: len(per.get((n, "TCC_MISS"), {})))  # the SpMV kernel (most dispatches)
    miss = per[(main, "TCC_MISS")]
    conf = per[(main, "SQ_LDS_BANK_CONFLICT")]
    assert int(rec["readMisses"]) == round(sum(miss.values()) / len(miss)), (main, rec["readMisses"])
    assert int(rec["hazardStalls"]) == round(sum(conf.values()) / len(conf)), (main, rec["hazardStalls"])
    assert "readMissesModel" in rec and "hazardStallsModel" in rec
