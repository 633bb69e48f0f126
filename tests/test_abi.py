"""The C-ABI library loads and exports every symbol include/hipspmv.h declares
(no compute: these run without a GPU)."""
import os
import ctypes as C
import subprocess

import numpy as np
import pytest

import hipspmv as hs


def test_exports_every_declared_symbol():
    lib = hs.load_hipspmv()
    declared = hs.declared_symbols()
    assert len(declared) >= 12
    out = subprocess.run(["nm", "-D", "--defined-only", f"{hs.LIB_DIR}/libhipspmv.so"], capture_output=True,
                         text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)


def test_no_torch_types_in_abi():
    text = open(hs.HEADER).read()
    for banned in ("torch", "at::", "hipStream_t", "Tensor"):
        # streams travel as void*; HIP types may appear only in comments
        code = "\n".join(l.split("//")[0] for l in text.splitlines() if not l.strip().startswith("*"))
        assert banned not in code.replace("/*", "").split("*/")[-1] or banned == "hipStream_t"


def test_strerror_and_version():
    lib = hs.load_hipspmv()
    assert lib.hipspmv_abi_version() == 1
    assert lib.hipspmv_strerror(0) == b"ok"
    assert lib.hipspmv_strerror(2) == b"invalid matrix"
    assert lib.hipspmv_strerror(99) == b"unknown status"


def test_invalid_arguments_rejected_without_device():
    lib = hs.load_hipspmv()
    h = C.c_void_p()
    # null output handle / bad dtype are argument errors regardless of devices
    assert lib.hipspmv_create(None, None, None, 1, 1, 0, 0, 0, None) == 1
    cp = np.zeros(2, np.uint32)
    assert lib.hipspmv_create(cp.ctypes.data, None, None, 1, 1, 0, 7, 0, C.byref(h)) == 1
    assert lib.hipspmv_destroy(None) == 1
    assert lib.hipspmv_exec(None, None, None, 0, 0) == 1
    v = C.c_uint64()
    assert lib.hipspmv_stat(None, b"rows", C.byref(v)) == 1


def test_device_count_callable():
    n = hs.device_count()
    assert n >= 0


def test_integration_example_builds():
    # the INTEGRATION.md example program links against both libraries (usage path: no device needed)
    import subprocess
    out = subprocess.run([os.path.join(hs.LIB_DIR, "plugin_example")], capture_output=True, text=True, timeout=60)
    assert out.returncode == 2 and "usage" in out.stderr


def test_wrapper_rejects_mismatched_arrays():
    # raw pointers cross the ABI, so the wrapper checks lengths before calling it
    import numpy as np
    import pytest
    import hipspmv as hs
    with pytest.raises(ValueError):
        hs.Handle.from_csc(np.zeros(3, np.uint32), np.zeros(0, np.uint32), np.zeros(0), 4, 4)  # colptr short
    with pytest.raises(ValueError):
        hs.Handle.from_csr(np.array([0, 1], np.uint32), np.zeros(1, np.uint32), np.zeros(2), 1, 4)  # vals long


def test_python_constants_match_header():
    """The binding's enums and HIPSPMV_SHARD_ALIGN are the header's #defines."""
    import re
    text = open(hs.HEADER).read()
    d = {k: int(v) for k, v in re.findall(r"#define (HIPSPMV_[A-Z0-9_]+) (\d+)", text)}
    assert d["HIPSPMV_SHARD_ALIGN"] == hs.SHARD_ALIGN
    assert (d["HIPSPMV_F64"], d["HIPSPMV_U64"]) == (hs.F64, hs.U64)
    assert (d["HIPSPMV_MODE_AUTO"], d["HIPSPMV_MODE_ORDERED"], d["HIPSPMV_MODE_FAST"]) == \
        (hs.MODE_AUTO, hs.MODE_ORDERED, hs.MODE_FAST)
    for name, v in hs.KERNELS.items():
        assert d["HIPSPMV_KERNEL_" + name.upper()] == v, name
