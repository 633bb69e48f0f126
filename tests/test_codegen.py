"""Machine-code checks on the gfx950 code objects inside libhipspmv.so (CPU only).

ORDERED mode's bit-exactness vs SoftwareSpMV (software/SoftwareSpMV.cpp:62,
`m_y[r] += a * x`, product rounded before the add) requires that no f64 FMA is
emitted in any kernel, and the north star rules out MFMA for this
memory-bound path.  Both are properties of the compiled code, checked here by
disassembling the offload bundles of the built library."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG

LIBDIR = os.path.join(PKG, "lib")

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tool(name):
    p = os.path.join(LLVM, name)
    if not os.path.exists(p):
        pytest.skip(f"{name} not in {LLVM}")
    return p


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    lib = os.path.join(LIBDIR, "libhipspmv.so")
    assert os.path.exists(lib), "libhipspmv.so not built"
    d = tmp_path_factory.mktemp("coobj")
    fat = d / "fat.bin"
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib, str(d / "stripped.so")],
                   check=True)
    blob = fat.read_bytes()
    offs = []
    i = blob.find(MAGIC)
    while i >= 0:
        offs.append(i)
        i = blob.find(MAGIC, i + 1)
    assert offs, "no offload bundle in .hip_fatbin"
    texts = []
    for k, o in enumerate(offs):
        e = offs[k + 1] if k + 1 < len(offs) else len(blob)
        b = d / f"b{k}.bin"
        b.write_bytes(blob[o:e])
        co = d / f"co{k}.o"
        subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        f"--targets={TARGET}", f"--output={co}"], check=True)
        if co.stat().st_size == 0:
            continue
        out = subprocess.run([_tool("llvm-objdump"), "-d", "-t", str(co)], check=True, capture_output=True,
                             text=True).stdout
        texts.append(out)
    assert texts, "no gfx950 code object in libhipspmv.so"
    return "\n".join(texts)


def test_kernels_present(disasm):
    for k in ("k_vcache", "k_csr_lane", "k_csr_vector", "k_sell", "k_wgather", "k_first_last", "k_alive_blocks"):
        assert k in disasm, k


def test_no_f64_fma(disasm):
    for op in ("v_fma_f64", "v_fmac_f64", "v_pk_fma_f64"):
        assert op not in disasm, f"{op} emitted: products must be rounded before the add"
    assert "v_mul_f64" in disasm and "v_add_f64" in disasm


def test_no_mfma(disasm):
    assert "v_mfma" not in disasm
