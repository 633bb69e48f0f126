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
        notes = subprocess.run([_tool("llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        texts.append(out + "\n" + notes)
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


def _kernel_notes(disasm):
    """(name, fields) for every kernel in the code-object metadata notes."""
    import re
    out = []
    for blk in re.split(r"\n\s+- \.agpr_count", disasm)[1:]:
        f = dict(re.findall(r"\.([a-z_]+):\s+(\S+)", blk))
        if "name" in f and "group_segment_fixed_size" in f:
            out.append((f["name"], f))
    return out


def test_kernel_resources_within_gfx950_limits(disasm):
    """Every kernel launches as compiled: LDS within the CU's 160 KiB, no
    scratch and no spills, and enough VGPRs free for its largest workgroup to
    be resident on one CU (4 SIMDs, 512 VGPRs per lane each)."""
    ks = _kernel_notes(disasm)
    assert len(ks) >= 20, len(ks)
    for name, f in ks:
        assert int(f["group_segment_fixed_size"]) <= 160 * 1024, name
        assert int(f["private_segment_fixed_size"]) == 0, name
        assert int(f["vgpr_spill_count"]) == 0 and int(f["sgpr_spill_count"]) == 0, name
        assert f.get("uses_dynamic_stack", "false") == "false", name
        waves_per_simd = -(-int(f["max_flat_workgroup_size"]) // 64 // 4)
        alloc = -(-(int(f["vgpr_count"]) + int(f.get("agpr_count", 0) or 0)) // 8) * 8
        assert alloc * waves_per_simd <= 512, (name, alloc, waves_per_simd)


def test_product_kernels_are_the_gpu_validated_machine_code():
    """The kernels AUTO selects (vcache split, sell, wgather, csr_vector; with
    vcache ordered and csr_lane; f64 and u64) compile to exactly the instructions of the last build that
    passed `pytest -m gpu` on an MI355X (tests/golden/validated_isa.json,
    recorded on the GPU box by tools/record_validated.py from the library those
    tests loaded): the round-end bench runs that machine code."""
    import json
    import sys
    sys.path.insert(0, os.path.join(PKG, "tools"))
    import kernel_isa
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "validated_isa.json")))
    now = kernel_isa.fingerprints(os.path.join(LIBDIR, "libhipspmv.so"))
    base = {n[:n.index(">(") + 1] if ">(" in n else n: v for n, v in now.items()}
    assert len(ref["kernels"]) >= 8
    for k in ref["kernels"]:
        assert k["current"] in base, k["current"]
        assert base[k["current"]]["sha256"] == k["sha256"], f"{k['current']} differs from the validated build"
