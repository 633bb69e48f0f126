"""ctypes binding of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product.  Parity pinning is
described in oracle.h (reference golden.bin files and the frontend KATs).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_u32 = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f64 = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u64 = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_lib = None


def build() -> None:
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.oracle_spmv_csc_f64.argtypes = [C.c_uint32, _u32, _u32, _f64, _f64, _f64]
        L.oracle_spmv_csc_u64.argtypes = [C.c_uint32, _u32, _u32, _u64, _u64, _u64]
        L.oracle_csr2csc.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, _u32, _u32, C.c_void_p, _u32, _u32]
        L.oracle_mark_row_starts.argtypes = [C.c_uint32, C.c_uint32, _u32, C.c_int, C.c_int]
        L.oracle_max_alive.argtypes = [C.c_uint32, C.c_uint32, _u32]
        L.oracle_max_alive.restype = C.c_uint32
        L.oracle_max_col_span.argtypes = [C.c_uint32, _u32, _u32]
        L.oracle_max_col_span.restype = C.c_uint32
        L.oracle_clear_row_markings.argtypes = [C.c_uint32, _u32, C.c_uint32]
        L.oracle_time_spmv_csc_f64.argtypes = [C.c_uint32, C.c_uint32, _u32, _u32, _f64, _f64, _f64, C.c_int]
        L.oracle_time_spmv_csc_f64.restype = C.c_double
        L.oracle_time_spmv_csr_f64_mt.argtypes = [C.c_uint32, _u32, _u32, _f64, _f64, _f64, C.c_int, C.c_int]
        L.oracle_time_spmv_csr_f64_mt.restype = C.c_double
        for f in (L.oracle_spmv_csc_f64, L.oracle_spmv_csc_u64, L.oracle_csr2csc, L.oracle_mark_row_starts,
                  L.oracle_clear_row_markings):
            f.restype = None
        _lib = L
    return _lib


def spmv_csc(colptr, rowind, vals, x, y=None, rows=None):
    """SoftwareSpMV::exec restated: y += A*x (y zeros if None). Returns y."""
    cols = colptr.size - 1
    if vals.dtype == np.uint64:
        y = np.zeros(rows, dtype=np.uint64) if y is None else y
        lib().oracle_spmv_csc_u64(cols, colptr, rowind, vals, np.ascontiguousarray(x, dtype=np.uint64), y)
    else:
        y = np.zeros(rows, dtype=np.float64) if y is None else y
        lib().oracle_spmv_csc_f64(cols, colptr, rowind, vals, np.ascontiguousarray(x, dtype=np.float64), y)
    return y


def csr2csc(n_rows, n_cols, rowptr, colind, vals):
    """csr2csc.c restated; also CSC->CSR when called with swapped roles."""
    nnz = colind.size
    colptr = np.empty(n_cols + 1, dtype=np.uint32)
    rowind = np.empty(nnz, dtype=np.uint32)
    out = np.empty(nnz, dtype=vals.dtype if vals is not None else np.uint64)
    a = None if vals is None else np.ascontiguousarray(vals).ctypes.data
    lib().oracle_csr2csc(n_rows, n_cols, nnz, a, np.ascontiguousarray(colind, dtype=np.uint32),
                         np.ascontiguousarray(rowptr, dtype=np.uint32), out.ctypes.data if vals is not None else None,
                         rowind, colptr)
    return colptr, rowind, (out if vals is not None else None)


def time_spmv_csc_f64(colptr, rowind, vals, x, rows, reps):
    y = np.zeros(rows, dtype=np.float64)
    return lib().oracle_time_spmv_csc_f64(rows, colptr.size - 1, colptr, rowind, vals, x, y, reps), y


def time_spmv_csr_f64_mt(rowptr, colind, vals, x, reps, nthreads):
    """Row-parallel CSR baseline on nthreads threads: (mean s/exec, y)."""
    rows = rowptr.size - 1
    y = np.zeros(rows, dtype=np.float64)
    t = lib().oracle_time_spmv_csr_f64_mt(rows, np.ascontiguousarray(rowptr, dtype=np.uint32),
                                          np.ascontiguousarray(colind, dtype=np.uint32),
                                          np.ascontiguousarray(vals, dtype=np.float64),
                                          np.ascontiguousarray(x, dtype=np.float64), y, reps, nthreads)
    return t, y


def mark_row_starts(inds, rows, reverse=False, shift=31):
    """SparseMatrix::markRowStarts restated; returns a marked copy."""
    out = np.array(inds, dtype=np.uint32, copy=True)
    lib().oracle_mark_row_starts(rows, out.size, out, int(reverse), shift)
    return out


def max_alive(inds, rows):
    """SparseMatrix::maxAlive restated (on a copy: the reference marks A in place)."""
    out = np.array(inds, dtype=np.uint32, copy=True)
    return int(lib().oracle_max_alive(rows, out.size, out))


def max_col_span(colptr, inds):
    """SparseMatrix::maxColSpan restated."""
    colptr = np.ascontiguousarray(colptr, dtype=np.uint32)
    return int(lib().oracle_max_col_span(colptr.size - 1, colptr, np.ascontiguousarray(inds, dtype=np.uint32)))
