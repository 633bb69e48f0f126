"""Python binding of the MI355X SpMV backend (ctypes over the C ABI).

Thin plumbing for bench.py and tests/: the product is libhipspmv.so (HIP
kernels + include/hipspmv.h) and libspmvhost.so (the C++ restatement of the
reference plugin surface).  This module only marshals numpy arrays / torch
tensors into the C ABI.  There is no CPU fallback: if the shared libraries
are missing, ``load_hipspmv`` raises.

PyTorch is imported first on purpose: it loads its HIP runtime
(libamdhip64.so.7) and libhipspmv.so, which needs the same soname, then binds
to that one instance, so device pointers and streams are shared.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess
import weakref

import numpy as np

try:  # torch first (see module docstring); absent torch is fine for host-only use
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
REPO_DIR = os.path.dirname(PKG_DIR)
HEADER = os.path.join(REPO_DIR, "include", "hipspmv.h")

F64, U64 = 0, 1
MODE_AUTO, MODE_ORDERED, MODE_FAST = 0, 1, 2
KERNEL_AUTO, KERNEL_VCACHE, KERNEL_CSR_LANE, KERNEL_CSR_VECTOR, KERNEL_VCACHE_SPLIT = 0, 1, 2, 3, 4
KERNEL_VCACHE_SPLIT4, KERNEL_WGATHER = 5, 6  # experimental: never chosen by AUTO
KERNEL_SELL = 7  # SELL-C-sigma lane per row
KERNEL_WCSR = 8  # csr_vector over column-windowed row segments + a window-order reduce (FAST)
KERNEL_VFLOW = 9  # four-part vector cache, x ring handed over by LDS flags (FAST, csrc/vflow.hip)
KERNEL_WGATHER_SPLIT = 10  # k_wgather over two column halves, one per XCD half, y = p0 + p1 (FAST)
SHARD_ALIGN = 64  # HIPSPMV_SHARD_ALIGN: row shards starting at multiples keep every kernel's bits
#                   (except WCSR in FAST f64: within the bound, not bit-identical; include/hipspmv.h)
KERNELS = {"auto": KERNEL_AUTO, "vcache": KERNEL_VCACHE, "csr_lane": KERNEL_CSR_LANE,
           "csr_vector": KERNEL_CSR_VECTOR, "vcache_split": KERNEL_VCACHE_SPLIT,
           "vcache_split4": KERNEL_VCACHE_SPLIT4, "wgather": KERNEL_WGATHER, "sell": KERNEL_SELL,
           "wcsr": KERNEL_WCSR, "vcache_flow": KERNEL_VFLOW, "wgather_split": KERNEL_WGATHER_SPLIT}
STATUS = {0: "ok", 1: "invalid argument", 2: "invalid matrix", 3: "HIP error", 4: "out of memory",
          5: "unsupported", 6: "no device", 7: "unknown key"}

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")

_hip = None
_host = None


class HipSpMVError(RuntimeError):
    def __init__(self, status: int, what: str):
        detail = ""
        if _hip is not None:
            detail = _hip.hipspmv_last_error().decode(errors="replace")
        super().__init__(f"{what}: {STATUS.get(status, status)}" + (f" ({detail})" if detail else ""))
        self.status = status


def build(force: bool = False) -> None:
    """Compile libhipspmv.so / libspmvhost.so / spmvbench in-tree (make)."""
    libs = [os.path.join(LIB_DIR, n) for n in ("libhipspmv.so", "libspmvhost.so", "spmvbench")]
    if force or not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-C", PKG_DIR, "-j8"], check=True)


class PrepStats(C.Structure):
    """hipspmv_prep_stats_t (include/hipspmv.h)"""
    _fields_ = [("max_alive", C.c_uint32), ("max_col_span", C.c_uint32), ("max_alive_ns", C.c_uint64),
                ("max_col_span_ns", C.c_uint64), ("cms_ns", C.c_uint64), ("h2d_ns", C.c_uint64)]


def declared_symbols() -> list[str]:
    """Function names declared in include/hipspmv.h."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(hipspmv_[a-z_0-9]+)\s*\(", text)))


def load_hipspmv() -> C.CDLL:
    global _hip
    if _hip is not None:
        return _hip
    # HIPSPMV_EXPERIMENTAL=1: the build with every kernel form (make EXPERIMENTAL=1), else the product
    exp = os.environ.get("HIPSPMV_EXPERIMENTAL") == "1"
    path = os.path.join(LIB_DIR, "exp", "libhipspmv.so") if exp else os.path.join(LIB_DIR, "libhipspmv.so")
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: build with `make -C {PKG_DIR}{' EXPERIMENTAL=1' if exp else ''}` "
                                "(no CPU fallback exists)")
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    vp = C.c_void_p
    lib.hipspmv_create.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.POINTER(vp)]
    lib.hipspmv_create_csr.argtypes = lib.hipspmv_create.argtypes
    lib.hipspmv_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    lib.hipspmv_exec.argtypes = [vp, vp, vp, C.c_int, C.c_int]
    lib.hipspmv_exec_device.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, vp]
    lib.hipspmv_stat.argtypes = [vp, C.c_char_p, C.POINTER(C.c_uint64)]
    lib.hipspmv_kernel_name.argtypes = [vp, C.c_int]
    lib.hipspmv_kernel_name.restype = C.c_char_p
    lib.hipspmv_destroy.argtypes = [vp]
    lib.hipspmv_release_wait.argtypes = []
    lib.hipspmv_build_flags.argtypes = []
    lib.hipspmv_pmc_counter.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint64)]
    lib.hipspmv_attach_pmc.argtypes = [vp, C.c_char_p]
    lib.hipspmv_strerror.argtypes = [C.c_int]
    lib.hipspmv_strerror.restype = C.c_char_p
    lib.hipspmv_last_error.argtypes = []
    lib.hipspmv_last_error.restype = C.c_char_p
    lib.hipspmv_abi_version.argtypes = []
    lib.hipspmv_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.hipspmv_prep_stats.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                       C.POINTER(PrepStats)]
    lib.hipspmv_mark_row_starts.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                            C.POINTER(C.c_uint64)]
    ip = C.POINTER(C.c_int)
    lib.hipspmv_multi_create.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, ip, C.c_int,
                                         C.POINTER(vp)]
    lib.hipspmv_multi_create_csr.argtypes = lib.hipspmv_multi_create.argtypes
    lib.hipspmv_multi_shard.argtypes = [vp, C.c_int, C.POINTER(vp)]
    lib.hipspmv_partition_rows.argtypes = [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp]
    lib.hipspmv_stream_bandwidth.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double),
                                             C.POINTER(C.c_double)]
    lib.hipspmv_multi_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    lib.hipspmv_multi_exec.argtypes = [vp, vp, vp, C.c_int, C.c_int]
    lib.hipspmv_multi_stat.argtypes = [vp, C.c_char_p, C.POINTER(C.c_uint64)]
    lib.hipspmv_multi_destroy.argtypes = [vp]
    for name in ("hipspmv_stream_bandwidth", "hipspmv_multi_create", "hipspmv_multi_create_csr", "hipspmv_multi_shard", "hipspmv_partition_rows",
                 "hipspmv_multi_set_option", "hipspmv_multi_exec", "hipspmv_multi_stat", "hipspmv_multi_destroy"):
        getattr(lib, name).restype = C.c_int
    for name in ("hipspmv_create", "hipspmv_create_csr", "hipspmv_set_option", "hipspmv_exec",
                 "hipspmv_exec_device", "hipspmv_stat", "hipspmv_destroy", "hipspmv_release_wait", "hipspmv_build_flags", "hipspmv_abi_version",
                 "hipspmv_device_count", "hipspmv_prep_stats", "hipspmv_mark_row_starts"):
        getattr(lib, name).restype = C.c_int
    _hip = lib
    return lib


def load_host() -> C.CDLL:
    global _host
    if _host is not None:
        return _host
    load_hipspmv()
    path = os.path.join(LIB_DIR, "libspmvhost.so")
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: build with `make -C {PKG_DIR}`")
    lib = C.CDLL(path)
    lib.spmvhost_gen_stripe_csr.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                            C.c_uint64, _u32p, _u32p, _f64p]
    lib.spmvhost_gen_stripe_csr.restype = None
    lib.spmvhost_gen_vector.argtypes = [C.c_uint64, C.c_uint64, _f64p]
    lib.spmvhost_gen_vector.restype = None
    lib.spmvhost_splitmix64_at.argtypes = [C.c_uint64, C.c_uint64]
    lib.spmvhost_splitmix64_at.restype = C.c_uint64
    lib.spmvhost_gen_rmat_csr.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, _u32p, _u32p, _f64p]
    lib.spmvhost_gen_rmat_csr.restype = C.c_uint64
    lib.spmvhost_gen_rmat_rows.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, _u32p, _u32p,
                                           _f64p, C.c_uint64]
    lib.spmvhost_gen_rmat_rows.restype = C.c_uint64
    lib.spmvhost_gen_rmat_row_counts.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, _u32p]
    lib.spmvhost_gen_rmat_row_counts.restype = None
    lib.spmvhost_partition_row_counts.argtypes = [_u32p, C.c_uint32, C.c_uint32, _u32p]
    lib.spmvhost_partition_row_counts.restype = None
    lib.spmvhost_csr2csc.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u64p, _u32p, _u32p, _u64p, _u32p, _u32p]
    lib.spmvhost_csr2csc.restype = None
    lib.spmvhost_partition_rows.argtypes = [_u32p, C.c_uint32, C.c_uint32, _u32p]
    lib.spmvhost_partition_rows.restype = None
    lib.spmvhost_load_matrix.argtypes = [C.c_char_p, C.c_char_p, _u32p, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.spmvhost_load_matrix.restype = C.c_int
    lib.spmvhost_convert_mtx.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    lib.spmvhost_row_len_histogram.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p, _u32p, _u32p,
                                               C.c_uint32]
    lib.spmvhost_row_len_histogram.restype = C.c_uint32
    lib.spmvhost_permute_longest_row_first.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, _u32p, _u32p, _u64p,
                                                       _u32p, _u32p, _u32p, _u64p]
    lib.spmvhost_permute_longest_row_first.restype = None
    lib.spmvhost_convert_mtx.restype = C.c_int
    _host = lib
    return lib


def _check(status: int, what: str) -> None:
    if status != 0:
        raise HipSpMVError(status, what)


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


class Handle:
    """One matrix resident on one device (a `hipspmv_t`)."""

    def __init__(self, ptr, ind, vals, rows: int, cols: int, *, csr: bool = False, device: int = 0):
        lib = load_hipspmv()
        ptr = np.ascontiguousarray(ptr, dtype=np.uint32)
        ind = np.ascontiguousarray(ind, dtype=np.uint32)
        if vals.dtype == np.uint64:
            self.dtype = U64
        elif vals.dtype == np.float64:
            self.dtype = F64
        else:
            raise TypeError("values must be float64 or uint64")
        vals = np.ascontiguousarray(vals)
        if ptr.size != (rows if csr else cols) + 1 or vals.size != ind.size:
            raise ValueError(f"{'rowptr' if csr else 'colptr'} needs {(rows if csr else cols) + 1} entries "
                             f"(got {ptr.size}) and one value per index (got {vals.size} for {ind.size})")
        self.rows, self.cols, self.nnz = int(rows), int(cols), int(ind.size)
        self.device = device
        h = C.c_void_p()
        fn = lib.hipspmv_create_csr if csr else lib.hipspmv_create
        _check(fn(ptr.ctypes.data, ind.ctypes.data, vals.ctypes.data, self.rows, self.cols, self.nnz,
                  self.dtype, device, C.byref(h)), "hipspmv_create")
        self._h = h
        self._lib = lib

    @classmethod
    def from_csc(cls, colptr, rowind, vals, rows, cols, device=0):
        return cls(colptr, rowind, vals, rows, cols, csr=False, device=device)

    @classmethod
    def from_csr(cls, rowptr, colind, vals, rows, cols, device=0):
        return cls(rowptr, colind, vals, rows, cols, csr=True, device=device)

    def set_option(self, key: str, value: int) -> None:
        _check(self._lib.hipspmv_set_option(self._handle(), key.encode(), int(value)), f"set_option({key})")

    def set_kernel(self, name: str) -> None:
        self.set_option("kernel", KERNELS[name])

    def kernel_name(self, mode: int = MODE_AUTO) -> str:
        return self._lib.hipspmv_kernel_name(self._handle(), mode).decode()

    def exec(self, x: np.ndarray, y: np.ndarray | None = None, beta: int = 0, mode: int = MODE_ORDERED):
        """Host-buffer exec (synchronous); returns y."""
        npdt = np.uint64 if self.dtype == U64 else np.float64
        x = np.ascontiguousarray(x, dtype=npdt)
        if y is None:
            y = np.zeros(self.rows, dtype=npdt)
        if x.size != self.cols or y.size != self.rows or y.dtype != npdt or not y.flags.c_contiguous:
            raise ValueError(f"x needs {self.cols} and y {self.rows} contiguous {np.dtype(npdt).name} elements")
        _check(self._lib.hipspmv_exec(self._handle(), x.ctypes.data, y.ctypes.data, beta, mode), "hipspmv_exec")
        return y

    def exec_device(self, x, y_out, y_in=None, beta: int = 0, mode: int = MODE_ORDERED, stream=None) -> None:
        """Device-tensor exec, enqueued on `stream` (torch stream or raw handle int)."""
        s = stream
        if s is not None and hasattr(s, "cuda_stream"):
            s = s.cuda_stream
        # the C ABI takes raw pointers: a short or strided tensor would be read
        # past its end on the device, so shapes are checked here
        for name, t, n in (("x", x, self.cols), ("y_out", y_out, self.rows), ("y_in", y_in, self.rows)):
            if t is None:
                continue
            if hasattr(t, "is_contiguous"):
                ok = (t.numel() == n and t.is_contiguous() and t.element_size() == 8 and t.is_cuda
                      and t.device.index == self.device)
            else:
                ok = False
            if not ok:
                raise ValueError(f"{name}: needs a contiguous 8-byte tensor of {n} elements on cuda:{self.device}")
        yin = _ptr(y_in) if y_in is not None else None
        _check(self._lib.hipspmv_exec_device(self._handle(), _ptr(x), yin, _ptr(y_out), beta, mode, s),
               "hipspmv_exec_device")

    def stat(self, key: str) -> int:
        v = C.c_uint64()
        _check(self._lib.hipspmv_stat(self._handle(), key.encode(), C.byref(v)), f"stat({key})")
        return int(v.value)

    def attach_pmc(self, csv_path: str | None) -> None:
        """A rocprofv3 --pmc counter CSV of this handle's kernel backs read_misses /
        hazard_stalls / capacity_stalls (include/hipspmv.h); None detaches."""
        _check(self._lib.hipspmv_attach_pmc(self._handle(), (csv_path or "").encode()), "attach_pmc")

    @classmethod
    def _borrowed(cls, h, rows: int, cols: int, nnz: int, dtype: int, device: int, parent):
        """A view of a handle owned elsewhere (a MultiHandle block): never destroyed
        here.  It keeps its parent alive, and the parent's close() invalidates it
        (a later call raises instead of reaching freed native memory)."""
        self = cls.__new__(cls)
        self.rows, self.cols, self.nnz, self.dtype, self.device = rows, cols, nnz, dtype, device
        self._h, self._lib, self._owner, self._parent = h, load_hipspmv(), False, parent
        return self

    def _handle(self):
        if not getattr(self, "_h", None):
            raise HipSpMVError(1, "handle closed (or its MultiHandle was)")
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None):
            if getattr(self, "_owner", True):
                self._lib.hipspmv_destroy(self._h)
            self._h = None
            self._parent = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prep_stats(colptr: np.ndarray, rowind: np.ndarray, rows: int, device: int = 0) -> dict:
    """SoftwareSpMV::measurePreprocessingTimes on the GPU (hipspmv_prep_stats):
    maxAlive, maxColSpan and the GPU times of the three scans, for a CSC matrix."""
    colptr = np.ascontiguousarray(colptr, dtype=np.uint32)
    rowind = np.ascontiguousarray(rowind, dtype=np.uint32)
    out = PrepStats()
    _check(load_hipspmv().hipspmv_prep_stats(_ptr(colptr), _ptr(rowind), rows, colptr.size - 1, rowind.size,
                                             device, C.byref(out)), "prep_stats")
    return {f: getattr(out, f) for f, _ in PrepStats._fields_}


def mark_row_starts(rowind: np.ndarray, rows: int, reverse: bool = False, shift: int = 31, device: int = 0):
    """SparseMatrix::markRowStarts on the GPU; returns (marked copy, kernel ns)."""
    rowind = np.ascontiguousarray(rowind, dtype=np.uint32)
    out = np.empty_like(rowind)
    ns = C.c_uint64()
    _check(load_hipspmv().hipspmv_mark_row_starts(_ptr(rowind), _ptr(out), rows, rowind.size, int(reverse), shift,
                                                  device, C.byref(ns)), "mark_row_starts")
    return out, int(ns.value)


class MultiHandle:
    """One matrix row-partitioned over several devices of this process
    (`hipspmv_multi_t`): x broadcast device to device, one block per device.
    CSC input (SparseMatrix) by default, CSR with csr=True."""

    def __init__(self, ptr, ind, vals, rows: int, cols: int, devices, *, csr: bool = False):
        lib = load_hipspmv()
        self._keep = [np.ascontiguousarray(ptr, dtype=np.uint32), np.ascontiguousarray(ind, dtype=np.uint32),
                      np.ascontiguousarray(vals)]
        if self._keep[0].size != (rows if csr else cols) + 1 or self._keep[2].size != self._keep[1].size:
            raise ValueError(f"{'rowptr needs rows' if csr else 'colptr needs cols'} + 1 entries and one value "
                             "per index")
        if self._keep[2].dtype not in (np.float64, np.uint64):
            raise TypeError("values must be float64 or uint64")
        self.dtype = self._keep[2].dtype
        self.rows, self.cols = rows, cols
        self.devices = list(devices)
        devs = (C.c_int * len(devices))(*devices)
        self._h = C.c_void_p()
        fn = lib.hipspmv_multi_create_csr if csr else lib.hipspmv_multi_create
        _check(fn(_ptr(self._keep[0]), _ptr(self._keep[1]), _ptr(self._keep[2]), rows, cols,
                  self._keep[1].size, U64 if self.dtype == np.uint64 else F64, devs,
                  len(devices), C.byref(self._h)), "multi_create")
        self._keep = None
        self._views = []  # borrowed shard Handles, invalidated by close()

    def shard(self, i: int):
        """Block i's own Handle (owned by this MultiHandle; None for a block without rows)."""
        h = C.c_void_p()
        _check(load_hipspmv().hipspmv_multi_shard(self._h, i, C.byref(h)), "multi_shard")
        if not h.value:
            return None
        sh = Handle._borrowed(h, self.stat(f"shard{i}_rows"), self.cols, self.stat(f"shard{i}_nz"),
                              U64 if self.dtype == np.uint64 else F64, self.devices[i], self)
        self._views.append(weakref.ref(sh))
        return sh

    def set_option(self, key: str, value: int) -> None:
        _check(load_hipspmv().hipspmv_multi_set_option(self._h, key.encode(), value), f"multi_set_option({key})")

    def set_kernel(self, name: str) -> None:
        self.set_option("kernel", KERNELS[name])

    def exec(self, x: np.ndarray, y: np.ndarray | None = None, beta: int = 0, mode: int = MODE_ORDERED):
        x = np.ascontiguousarray(x, dtype=self.dtype)
        y = np.zeros(self.rows, dtype=self.dtype) if y is None else np.ascontiguousarray(y, dtype=self.dtype)
        if x.size != self.cols or y.size != self.rows:
            raise ValueError(f"x needs {self.cols} and y {self.rows} elements")
        _check(load_hipspmv().hipspmv_multi_exec(self._h, _ptr(x), _ptr(y), beta, mode), "multi_exec")
        return y

    def stat(self, key: str) -> int:
        v = C.c_uint64()
        _check(load_hipspmv().hipspmv_multi_stat(self._h, key.encode(), C.byref(v)), f"multi_stat({key})")
        return int(v.value)

    def close(self) -> None:
        for ref in getattr(self, "_views", []):
            sh = ref()
            if sh is not None:
                sh._h = None
        self._views = []
        if self._h:
            load_hipspmv().hipspmv_multi_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stream_bandwidth(device: int = 0, nbytes: int = 1 << 30, reps: int = 10) -> tuple:
    """(copy GB/s counting read + write, read GB/s) of the in-tree streaming
    kernels on buffers of nbytes (hipspmv_stream_bandwidth): the measured HBM
    ceiling bench.py reports beside the 8 TB/s roofline."""
    cp, rd = C.c_double(), C.c_double()
    _check(load_hipspmv().hipspmv_stream_bandwidth(device, nbytes, reps, C.byref(cp), C.byref(rd)), "stream_bandwidth")
    return float(cp.value), float(rd.value)


def device_count() -> int:
    n = C.c_int()
    _check(load_hipspmv().hipspmv_device_count(C.byref(n)), "device_count")
    return int(n.value)


# ---------------------------------------------------------------- host helpers
def gen_stripe_csr(row0: int, nrows: int, cols: int, k: int = 32, seed_col: int = 1, seed_val: int = 2):
    lib = load_host()
    rowptr = np.empty(nrows + 1, dtype=np.uint32)
    colind = np.empty(nrows * k, dtype=np.uint32)
    vals = np.empty(nrows * k, dtype=np.float64)
    lib.spmvhost_gen_stripe_csr(row0, nrows, cols, k, seed_col, seed_val, rowptr, colind, vals)
    return rowptr, colind, vals


def gen_vector(n: int, seed: int = 3) -> np.ndarray:
    out = np.empty(n, dtype=np.float64)
    load_host().spmvhost_gen_vector(n, seed, out)
    return out


def gen_rmat_csr(scale: int, edge_factor: int = 16, seed: int = 4):
    lib = load_host()
    n, m = 1 << scale, edge_factor << scale
    rowptr = np.empty(n + 1, dtype=np.uint32)
    colind = np.empty(m, dtype=np.uint32)
    vals = np.empty(m, dtype=np.float64)
    nnz = lib.spmvhost_gen_rmat_csr(scale, edge_factor, seed, rowptr, colind, vals)
    return rowptr, colind[:nnz].copy(), vals[:nnz].copy()


def pmc_counter(csv_path: str, counter: str, kernel: str | None = None):
    """(mean per dispatch, dispatches) of `counter` in a rocprofv3 --pmc CSV over the
    dispatches whose kernel name contains `kernel` (hipspmv_pmc_counter; no GPU needed)."""
    m, n = C.c_double(), C.c_uint64()
    _check(load_hipspmv().hipspmv_pmc_counter(csv_path.encode(), kernel.encode() if kernel else None,
                                              counter.encode(), C.byref(m), C.byref(n)), f"pmc_counter({counter})")
    return float(m.value), int(n.value)


def gen_rmat_row_counts(scale: int, edge_factor: int = 16, seed: int = 4) -> np.ndarray:
    counts = np.empty(1 << scale, dtype=np.uint32)
    load_host().spmvhost_gen_rmat_row_counts(scale, edge_factor, seed, counts)
    return counts


def partition_row_counts(counts: np.ndarray, parts: int) -> np.ndarray:
    bounds = np.empty(parts + 1, dtype=np.uint32)
    load_host().spmvhost_partition_row_counts(np.ascontiguousarray(counts, dtype=np.uint32), counts.size, parts, bounds)
    return bounds


def rmat_expected_segments(counts: np.ndarray, scale: int, log2w: int = 20, a: float = 0.57, b: float = 0.19,
                           c: float = 0.19, cap: int = 256) -> np.ndarray:
    """Expected wcsr segments per row of the R-MAT matrix gen_rmat_rows makes
    (DESIGN.md §6.11): a row of len edges, whose columns are independent given
    the row (every level of host/Synthetic.cpp rmatEdge picks the column bit
    with P(1 | row bit 0) = b / (a + b), P(1 | row bit 1) = d / (c + d)),
    touches window w (the top scale - log2w column bits) with probability
    p_w(row) = prod_k P(col bit k | row bit k), so E[windows] =
    sum_w 1 - (1 - p_w)^len; pieces past `cap` entries in a window add
    max(0, len * p_w - cap) / cap.  Depends on the row only through its top
    scale - log2w bits and its length."""
    d = 1.0 - a - b - c
    k = max(0, scale - log2w)
    nw = 1 << k
    p1 = (b / (a + b), d / (c + d))  # P(col bit = 1 | row bit 0 / 1)
    counts = np.asarray(counts, dtype=np.int64)
    rows = counts.size
    prefix = (np.arange(rows, dtype=np.int64) >> (scale - k)) if k else np.zeros(rows, np.int64)
    wbits = (np.arange(nw)[:, None] >> (k - 1 - np.arange(k))[None, :]) & 1 if k else np.zeros((1, 0), np.int64)
    out = np.zeros(rows, dtype=np.float64)
    for pf in range(1 << k):
        rbits = (pf >> (k - 1 - np.arange(k))) & 1 if k else np.zeros(0, np.int64)
        q = np.array([p1[r] for r in rbits]) if k else np.zeros(0)
        pw = np.prod(np.where(wbits == 1, q[None, :], 1.0 - q[None, :]), axis=1) if k else np.ones(1)
        sel = np.nonzero(prefix == pf)[0]
        lens, inv = np.unique(counts[sel], return_inverse=True)
        L = lens.astype(np.float64)[:, None]
        e = np.sum(1.0 - np.power(1.0 - pw[None, :], L), axis=1) + \
            np.sum(np.maximum(0.0, L * pw[None, :] - cap), axis=1) / cap
        out[sel] = e[inv]
    return out


def partition_row_weights(weights: np.ndarray, parts: int) -> np.ndarray:
    """Contiguous row partition balancing the sum of per-row weights (a cost
    model), interior bounds snapped to the nearer multiple of SHARD_ALIGN like
    host/Synthetic.cpp partitionRowCounts: bounds[0] = 0, bounds[parts] = rows."""
    w = np.asarray(weights, dtype=np.float64)
    rows = w.size
    cum = np.concatenate([[0.0], np.cumsum(w)])
    bounds = np.zeros(parts + 1, dtype=np.int64)
    for p in range(1, parts):
        r = int(np.searchsorted(cum, cum[-1] * p / parts, side="left"))
        r = min(r, rows)
        lo = r // SHARD_ALIGN * SHARD_ALIGN
        snapped = min(rows, lo if r - lo <= SHARD_ALIGN // 2 else lo + SHARD_ALIGN)
        bounds[p] = max(snapped, bounds[p - 1])
    bounds[parts] = rows
    return bounds.astype(np.uint32)


# wcsr shard cost per row in entry units: each segment and
# each row costs this many entries' time -- the least-squares fit (no
# intercept) of the eight per-shard kernel times of C5 at the library's
# window (kWcLog2Window = 20), round 4 (profiles/r04/logs/bench_c5_w20.log:
# 7.08 us per M entries, 6.77 per M segments, 7.51 per M rows; residuals
# within 3 us of 271-283)
WCSR_COST_SEGMENT, WCSR_COST_ROW = 0.956, 1.061


def c5_partition(scale: int, parts: int, edge_factor: int = 16, seed: int = 4, model: str = "cost"):
    """C5's row partition: "nnz" balances entries (partition_row_counts);
    "cost" balances entries + WCSR_COST_SEGMENT * expected segments +
    WCSR_COST_ROW per row.  Returns (bounds, per-row counts)."""
    counts = gen_rmat_row_counts(scale, edge_factor, seed)
    if model == "nnz":
        return partition_row_counts(counts, parts), counts
    segs = rmat_expected_segments(counts, scale)
    w = counts.astype(np.float64) + WCSR_COST_SEGMENT * segs + WCSR_COST_ROW
    return partition_row_weights(w, parts), counts


def gen_rmat_rows(scale: int, row0: int, row1: int, edge_factor: int = 16, seed: int = 4, cap: int | None = None):
    """Rows [row0, row1) of gen_rmat_csr(scale, ...), rowptr rebased to 0."""
    lib = load_host()
    nr = row1 - row0
    if cap is None:
        cap = edge_factor << scale if nr == (1 << scale) else int(gen_rmat_row_counts(scale, edge_factor, seed)[row0:row1].sum(dtype=np.uint64))
    rowptr = np.empty(nr + 1, dtype=np.uint32)
    colind = np.empty(max(cap, 1), dtype=np.uint32)
    vals = np.empty(max(cap, 1), dtype=np.float64)
    nnz = lib.spmvhost_gen_rmat_rows(scale, edge_factor, seed, row0, row1, rowptr, colind, vals, cap)
    if nnz > cap:
        raise RuntimeError(f"gen_rmat_rows: {nnz} nonzeros exceed the capacity {cap}")
    return rowptr, colind[:nnz].copy(), vals[:nnz].copy()


def csr2csc(rows: int, cols: int, rowptr, colind, vals):
    """Product transpose (libspmvhost csr2csc); 8-byte values moved as words."""
    lib = load_host()
    nnz = int(colind.size)
    v = np.ascontiguousarray(vals).view(np.uint64)
    colptr = np.empty(cols + 1, dtype=np.uint32)
    rowind = np.empty(nnz, dtype=np.uint32)
    out = np.empty(nnz, dtype=np.uint64)
    lib.spmvhost_csr2csc(rows, cols, nnz, v, np.ascontiguousarray(colind, dtype=np.uint32),
                         np.ascontiguousarray(rowptr, dtype=np.uint32), out, rowind, colptr)
    return colptr, rowind, out.view(vals.dtype)


def partition_rows_cost(rowptr: np.ndarray, colind: np.ndarray, cols: int, parts: int) -> np.ndarray:
    """The library's row partition (hipspmv_partition_rows, the one
    hipspmv_multi_create uses): cost-balanced contiguous blocks, a row costing
    entries + wcsr segments + 1; bounds[parts + 1] as uint32."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.uint32)
    colind = np.ascontiguousarray(colind, dtype=np.uint32)
    bounds = np.empty(parts + 1, dtype=np.uint32)
    _check(load_hipspmv().hipspmv_partition_rows(_ptr(rowptr), _ptr(colind), rowptr.size - 1, cols, parts,
                                                 _ptr(bounds)), "partition_rows")
    return bounds


def partition_rows(rowptr: np.ndarray, parts: int) -> np.ndarray:
    rows = rowptr.size - 1
    bounds = np.empty(parts + 1, dtype=np.uint32)
    load_host().spmvhost_partition_rows(np.ascontiguousarray(rowptr, dtype=np.uint32), rows, parts, bounds)
    return bounds


def load_matrix(directory: str, name: str):
    """(rows, cols, colptr, rowind, vals) of a reference-format matrix."""
    lib = load_host()
    dims = np.zeros(4, dtype=np.uint32)
    _check(lib.spmvhost_load_matrix(directory.encode(), name.encode(), dims, None, None, None), f"load {name}")
    rows, cols, nnz, is_u64 = (int(d) for d in dims)
    colptr = np.empty(cols + 1, dtype=np.uint32)
    rowind = np.empty(nnz, dtype=np.uint32)
    vals = np.empty(nnz, dtype=np.uint64)
    _check(lib.spmvhost_load_matrix(directory.encode(), name.encode(), dims, colptr.ctypes.data,
                                    rowind.ctypes.data, vals.ctypes.data), f"load {name}")
    return rows, cols, colptr, rowind, (vals if is_u64 else vals.view(np.float64))


def convert_mtx(mtx_path: str, outdir: str, name: str, golden: bool = True, permute: bool = False) -> None:
    """Matrix Market -> reference .bin layout (+ golden.bin) via libspmvhost;
    permute: rows longest first (matrixutils.py:149-158) before writing."""
    os.makedirs(os.path.join(outdir, name), exist_ok=True)
    _check(load_host().spmvhost_convert_mtx(mtx_path.encode(), outdir.encode(), name.encode(), int(golden),
                                            int(permute)), f"convert {mtx_path}")


def row_len_histogram(colptr, rowind, rows: int) -> dict:
    """generateRowLenHistogram (matrixutils.py:116-126) via libspmvhost."""
    colptr = np.ascontiguousarray(colptr, dtype=np.uint32)
    rowind = np.ascontiguousarray(rowind, dtype=np.uint32)
    cap = rows + 1
    lens, counts = np.empty(cap, np.uint32), np.empty(cap, np.uint32)
    n = load_host().spmvhost_row_len_histogram(rows, colptr.size - 1, rowind.size, colptr, rowind, lens, counts, cap)
    return {int(k): int(v) for k, v in zip(lens[:n], counts[:n])}


def permute_longest_row_first(colptr, rowind, vals, rows: int):
    """permuteLongestRowFirst (matrixutils.py:140-158): (perm, colptr, rowind, vals)."""
    colptr = np.ascontiguousarray(colptr, dtype=np.uint32)
    rowind = np.ascontiguousarray(rowind, dtype=np.uint32)
    vals = np.ascontiguousarray(vals)
    cols, nz = colptr.size - 1, rowind.size
    perm = np.empty(rows, np.uint32)
    cp, ri, v = np.empty(cols + 1, np.uint32), np.empty(nz, np.uint32), np.empty(nz, np.uint64)
    load_host().spmvhost_permute_longest_row_first(rows, cols, nz, colptr, rowind, vals.view(np.uint64), perm, cp,
                                                   ri, v)
    return perm, cp, ri, v.view(vals.dtype)


def release_wait() -> None:
    """Until every handle destroyed so far has had its device memory released
    (hipspmv_release_wait; destroy itself returns at once)."""
    _check(load_hipspmv().hipspmv_release_wait(), "release_wait")


def experimental_build() -> bool:
    """True when the loaded library carries the kernel forms AUTO never picks
    (hipspmv_build_flags; make EXPERIMENTAL=1, loaded under HIPSPMV_EXPERIMENTAL=1)."""
    return bool(load_hipspmv().hipspmv_build_flags() & 1)
