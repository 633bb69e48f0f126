#!/usr/bin/env python3
"""Per-kernel machine-code fingerprints of the gfx950 code objects in a built
libhipspmv.so.

Each kernel's disassembly is normalised -- addresses, encodings and branch
labels dropped, branch targets rewritten as offsets in instructions -- so two
builds of the same source give the same text regardless of where the linker
placed the function.  The fingerprint is the sha256 of that text; the kernel
key is its demangled name with the template arguments of the kernel as
compiled (trailing defaulted parameters of later source revisions are
reported separately by the caller).

    python tools/kernel_isa.py LIB.so [--json OUT]      # name -> {sha256, insts}
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _code_objects(lib, tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib,
                    os.path.join(tmp, "stripped.so")], check=True)
    blob = open(fat, "rb").read()
    offs = []
    i = blob.find(MAGIC)
    while i >= 0:
        offs.append(i)
        i = blob.find(MAGIC, i + 1)
    out = []
    for k, o in enumerate(offs):
        e = offs[k + 1] if k + 1 < len(offs) else len(blob)
        b = os.path.join(tmp, f"b{k}.bin")
        open(b, "wb").write(blob[o:e])
        co = os.path.join(tmp, f"co{k}.o")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                        f"--targets={TARGET}", f"--output={co}"], check=True)
        if os.path.getsize(co):
            out.append(co)
    return out


_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")


def _demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


def fingerprints(lib):
    """{demangled kernel name: {"sha256": ..., "insts": n}} for every kernel.
    Branch operands are instruction-relative (simm16) already, so dropping the
    `// address: encoding <symbol+off>` comment makes the text position-free."""
    funcs = {}
    with tempfile.TemporaryDirectory() as tmp:
        for co in _code_objects(lib, tmp):
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = _FUNC.match(line)
                if m:
                    cur = m.group(2)
                    funcs[cur] = []
                elif cur is not None and line.startswith("\t"):
                    inst = line.split("//")[0].strip()
                    if inst:
                        funcs[cur].append(" ".join(inst.split()))
    names = [k for k, v in funcs.items() if v and not k.endswith(".kd")]
    out = {}
    for mangled, dem in zip(names, _demangle(names)):
        text = "\n".join(funcs[mangled])
        out[dem] = {"sha256": hashlib.sha256(text.encode()).hexdigest(), "insts": len(funcs[mangled])}
    return out


def main(argv):
    lib = argv[1]
    fp = fingerprints(lib)
    if "--json" in argv:
        with open(argv[argv.index("--json") + 1], "w") as f:
            json.dump(fp, f, indent=1, sort_keys=True)
    for k in sorted(fp):
        print(f"{fp[k]['sha256'][:16]} {fp[k]['insts']:6d}  {k[:150]}")


if __name__ == "__main__":
    main(sys.argv)
