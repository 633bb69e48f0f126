"""Readers for the reference's fixture matrices (tests/golden/matrices, copied
verbatim from maltanar/spmv-vector-cache matrices/*/*.bin) using numpy only,
independent of the product loader."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MATRICES = os.path.join(GOLDEN, "matrices")
F64_FIXTURES = ["i64", "i1k", "i64k", "row64k", "circuit204"]
U64_FIXTURES = ["i64-uint64", "dia64-uint64", "rowvec64-uint64", "i1024-uint64", "circuit204-uint64"]
ALL_FIXTURES = F64_FIXTURES + U64_FIXTURES


def load(name):
    d = os.path.join(MATRICES, name)
    meta = np.fromfile(os.path.join(d, f"{name}-meta.bin"), dtype=np.uint32)
    rows, cols, nnz = (int(v) for v in meta[:3])
    colptr = np.fromfile(os.path.join(d, f"{name}-indptr.bin"), dtype=np.uint32)
    rowind = np.fromfile(os.path.join(d, f"{name}-inds.bin"), dtype=np.uint32)
    vals = np.fromfile(os.path.join(d, f"{name}-data.bin"), dtype=np.uint64 if "uint64" in name else np.float64)
    assert colptr.size == cols + 1 and rowind.size == nnz and vals.size == nnz
    return rows, cols, colptr, rowind, vals


def golden(name):
    p = os.path.join(MATRICES, name, "golden.bin")
    return np.fromfile(p, dtype=np.float64) if os.path.exists(p) else None


def x_variants(name, cols):
    """The input vectors parity is checked on: ones (main.cpp:217-219),
    1..n (TestSpMVFrontend.scala:129-131), seeded U[-1,1) (f64 only), and for
    u64 large values that wrap mod 2^64."""
    out = {"ones": np.ones(cols), "iota": np.arange(1, cols + 1, dtype=np.float64)}
    if "uint64" in name:
        out = {k: v.astype(np.uint64) for k, v in out.items()}
        rng = np.random.default_rng(7)
        out["wrap"] = rng.integers(0, 2**64, size=cols, dtype=np.uint64)
    else:
        out["rand"] = np.random.default_rng(7).uniform(-1, 1, cols)
    return out


def csc_to_dense(rows, cols, colptr, rowind, vals):
    A = np.zeros((rows, cols), dtype=vals.dtype)
    for c in range(cols):
        for e in range(colptr[c], colptr[c + 1]):
            A[rowind[e], c] += vals[e]
    return A
