"""Golden output vectors (tests/golden/vectors.json, made by
tests/golden/make_vectors.py from the oracle).

CPU: the oracle still reproduces every committed vector, and the product's
C++ generators (host/Synthetic.cpp, used by bench.py and the GPU tests)
produce exactly the numpy restatement's matrices and vectors.
GPU: the ordered kernels (and every u64 run) reproduce the committed digests
through the C ABI, independent of the oracle at run time; a row-partitioned
run is bit-identical to the unpartitioned one in both modes."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

import fixtures as fx
import hipspmv as hs
import oracle

sys.path.insert(0, fx.GOLDEN)
import make_vectors as mv  # noqa: E402
import synth_numpy as sn  # noqa: E402

with open(os.path.join(fx.GOLDEN, "vectors.json")) as _f:
    VEC = json.load(_f)


def sha(y: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(y).view(np.uint64).tobytes()).hexdigest()


def _fixture_cases():
    for name, ent in VEC["fixtures"].items():
        for case in ent["cases"]:
            yield name, case


def _inputs(name, case, cols, rows, u64):
    xk, b = case.split("/")
    beta = int(b[-1])
    return mv.x_input(xk, cols, u64), beta, (mv.y0_input(rows, u64) if beta else None)


# ------------------------------------------------------------------ CPU
def test_vectors_cover_all_fixtures():
    assert set(VEC["fixtures"]) == set(fx.ALL_FIXTURES)
    assert all(len(e["cases"]) == 6 for e in VEC["fixtures"].values())


@pytest.mark.parametrize("name", fx.ALL_FIXTURES)
def test_oracle_reproduces_fixture_vectors(name):
    rows, cols, colptr, rowind, vals = fx.load(name)
    u64 = vals.dtype == np.uint64
    for case, want in VEC["fixtures"][name]["cases"].items():
        x, beta, y0 = _inputs(name, case, cols, rows, u64)
        y = oracle.spmv_csc(colptr, rowind, vals, x, y=y0, rows=rows)
        assert sha(y) == want["sha256"], (name, case)


def test_x_ones_vectors_equal_reference_golden_bin():
    # the committed digest for x = ones, beta 0 is the reference's own golden.bin
    for name in fx.F64_FIXTURES:
        assert VEC["fixtures"][name]["cases"]["ones/beta0"]["sha256"] == sha(fx.golden(name)), name


@pytest.mark.parametrize("name", ["stripe_4096x4096_k32", "C3_rank1_shard_64Kx1M", "rmat_s14_ef16"])
def test_oracle_reproduces_synthetic_vectors(name):
    ent = VEC["synthetic"][name]
    rows, cols, rowptr, colind, vals = mv.synth_csr(ent["spec"])
    assert colind.size == ent["nnz"]
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    for case, want in ent["cases"].items():
        y = oracle.spmv_csc(colptr, rowind, cvals, mv.x_input(case.split("/")[0], cols, False), rows=rows)
        assert sha(y) == want["sha256"], (name, case)


def test_product_stripe_generator_matches_numpy():
    for row0, nrows, cols, k in [(0, 4096, 4096, 32), (1 << 20, 1024, 1 << 20, 32), (77, 300, 1000, 7),
                                 ((1 << 24) - 512, 512, 1 << 24, 32)]:
        a = hs.gen_stripe_csr(row0, nrows, cols, k)
        b = sn.stripe_csr(row0, nrows, cols, k)
        for u, v in zip(a, b):
            assert u.dtype == v.dtype and np.array_equal(u.view(np.uint64) if u.dtype == np.float64 else u,
                                                         v.view(np.uint64) if v.dtype == np.float64 else v)


def test_product_rmat_generator_matches_numpy():
    for scale in (8, 12):
        a = hs.gen_rmat_csr(scale, 16, 4)
        b = sn.rmat_csr(scale, 16, 4)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        assert a[2].tobytes() == b[2].tobytes()


def test_product_vector_generator_matches_numpy():
    assert hs.gen_vector(10000, 3).tobytes() == sn.vector_f64(10000, 3).tobytes()


# ------------------------------------------------------------------ GPU
ORDERED = ["vcache", "csr_lane", "sell"]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ORDERED + ["csr_vector", "vcache_split"])
def test_gpu_fixture_vectors(gpu, kernel):
    for name in fx.ALL_FIXTURES:
        rows, cols, colptr, rowind, vals = fx.load(name)
        u64 = vals.dtype == np.uint64
        if kernel not in ORDERED and not u64:
            continue  # FAST f64 kernels are checked against the bound elsewhere
        h = hs.Handle.from_csc(colptr, rowind, vals, rows, cols)
        if kernel.startswith("vcache") and not h.stat(
                "vcache_split_eligible" if kernel == "vcache_split" else "vcache_eligible"):
            h.close()
            continue
        h.set_kernel(kernel)
        mode = hs.MODE_ORDERED if kernel in ORDERED else hs.MODE_FAST
        for case, want in VEC["fixtures"][name]["cases"].items():
            x, beta, y0 = _inputs(name, case, cols, rows, u64)
            y = h.exec(x, y0, beta=beta, mode=mode)
            assert sha(y) == want["sha256"], (name, case, kernel)
        h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(VEC["synthetic"]))
def test_gpu_synthetic_vectors_ordered(gpu, name):
    ent = VEC["synthetic"][name]
    spec = ent["spec"]
    if spec["kind"] == "stripe":
        rowptr, colind, vals = hs.gen_stripe_csr(spec["row0"], spec["rows"], spec["cols"], spec["k"])
        rows, cols = spec["rows"], spec["cols"]
    else:
        rowptr, colind, vals = hs.gen_rmat_csr(spec["scale"], spec["edge_factor"], spec["seed"])
        rows = cols = 1 << spec["scale"]
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    for case, want in ent["cases"].items():
        y = h.exec(mv.x_input(case.split("/")[0], cols, False), beta=0, mode=hs.MODE_ORDERED)
        assert sha(y) == want["sha256"], (name, case, h.kernel_name(hs.MODE_ORDERED))
    h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,mode", [("auto", hs.MODE_ORDERED), ("vcache_split", hs.MODE_FAST),
                                         ("vcache", hs.MODE_ORDERED), ("sell", hs.MODE_FAST)])
def test_gpu_row_partition_bit_identical(gpu, kernel, mode):
    """Row shards (the multi-GPU layout) give bit-identical rows to one
    unpartitioned run: no arithmetic depends on where a shard starts."""
    rows, cols = 1 << 17, 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
    x = hs.gen_vector(cols, 3)
    whole = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    if kernel != "auto":
        whole.set_kernel(kernel)
    y = whole.exec(x, beta=0, mode=mode)
    whole.close()
    for parts in (2, 3):
        bounds = hs.partition_rows(rowptr, parts)
        for p in range(parts):
            r0, r1 = int(bounds[p]), int(bounds[p + 1])
            e0, e1 = int(rowptr[r0]), int(rowptr[r1])
            sh = hs.Handle.from_csr((rowptr[r0:r1 + 1] - rowptr[r0]).astype(np.uint32), colind[e0:e1],
                                    vals[e0:e1], r1 - r0, cols)
            if kernel != "auto":
                sh.set_kernel(kernel)
            ys = sh.exec(x, beta=0, mode=mode)
            sh.close()
            assert ys.tobytes() == y[r0:r1].tobytes(), (parts, p, kernel)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,mode", [("csr_vector", hs.MODE_FAST), ("sell", hs.MODE_FAST),
                                         ("csr_lane", hs.MODE_ORDERED), ("auto", hs.MODE_ORDERED)])
def test_gpu_row_partition_bit_identical_skewed(gpu, kernel, mode):
    """The same on R-MAT rows of very different lengths, where csr_vector's row
    groups differ from row to row: shards cut at multiples of
    HIPSPMV_SHARD_ALIGN (what partition_rows returns) keep the FAST bits of a
    given kernel.  (AUTO may pick a different FAST kernel for a smaller shard;
    in ORDERED mode every kernel gives the same bits.)"""
    n = 1 << 16
    rowptr, colind, vals = hs.gen_rmat_csr(16)
    x = hs.gen_vector(n, 3)
    whole = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    if kernel != "auto":
        whole.set_kernel(kernel)
    y = whole.exec(x, beta=0, mode=mode)
    whole.close()
    for parts in (2, 3, 5):
        bounds = hs.partition_rows(rowptr, parts)
        assert all(int(b) % 64 == 0 for b in bounds[1:-1])
        for p in range(parts):
            r0, r1 = int(bounds[p]), int(bounds[p + 1])
            if r1 == r0:
                continue
            e0, e1 = int(rowptr[r0]), int(rowptr[r1])
            sh = hs.Handle.from_csr((rowptr[r0:r1 + 1] - rowptr[r0]).astype(np.uint32), colind[e0:e1],
                                    vals[e0:e1], r1 - r0, n)
            if kernel != "auto":
                sh.set_kernel(kernel)
            ys = sh.exec(x, beta=0, mode=mode)
            sh.close()
            assert ys.tobytes() == y[r0:r1].tobytes(), (parts, p, kernel)
