#!/usr/bin/env python3
"""Record the machine-code fingerprints of the kernels AUTO can select, from
the libhipspmv.so a GPU session has just validated (tools/gpu_session.sh runs
this right after `pytest -m gpu` passes, on the box, over the library those
tests loaded).  The output replaces tests/golden/validated_isa.json when the
session is collected, so tests/test_codegen.py and bench.py's
kernel_provenance compare today's build with the last build that passed the
GPU tests.

    python tools/record_validated.py LIB.so OUT.json "pytest -m gpu: 230 passed (session log)"
"""
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_isa  # noqa: E402

# the instantiations choose_kernel (csrc/capi.cpp) can launch without options
PRODUCT = [f"void hipspmv::k_{k}<{t}{a}>" for t in ("double", "unsigned long")
           for k, a in (("vcache", ", 1, 8, 4, 3, 0, 0, false, 0, 0"), ("vcache", ", 3, 3, 4, 2, 0, 0, false, 1, 3"),
                        ("vcache", ", 3, 3, 4, 2, 0, 0, false, 1, 5"),
                        ("csr_lane", ""), ("csr_vector", ", false"), ("wgather", ", 16, 4, 2, true, true"), ("wgather", ", 16, 4, 3, true, true"),
                        ("wgather", ", 16, 2, 6, true, true"), ("wgather", ", 16, 2, 9, true, true"),
                        ("wgather", ", 16, 4, 2, true, false"),
                        ("wgather_split", ", 16, 4, 2, true, true"), ("wgather_split", ", 16, 4, 3, true, true"),
                        ("wgather_split", ", 16, 2, 6, true, true"), ("wgather_split", ", 16, 2, 9, true, true"),
                        ("wgather_split", ", 16, 4, 2, true, false"))] + \
          [f"void hipspmv::(anonymous namespace)::k_sell<{a}>" for a in
           ("double, true", "double, false", "unsigned long, false")] + \
          ["void hipspmv::(anonymous namespace)::k_sell_iso<45>"] + \
          [f"void hipspmv::k_{k}" for t in ("double", "unsigned long")
           for k in (f"csr_vector<{t}, true>", f"wreduce<{t}>")]


def main():
    lib, out, note = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""
    fps = kernel_isa.fingerprints(lib)
    base = {n[:n.index(">(") + 1] if ">(" in n else n: v for n, v in fps.items()}
    missing = [k for k in PRODUCT if k not in base]
    if missing:
        sys.exit(f"not in {lib}: {missing}")
    try:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                cwd=os.path.dirname(lib)).stdout.strip() or "n/a"
    except OSError:
        commit = "n/a"
    doc = {"about": ("Machine-code fingerprints (tools/kernel_isa.py: normalised llvm-objdump text of each gfx950 "
                     "kernel, sha256) of the kernels AUTO can select, recorded by tools/record_validated.py on the "
                     f"GPU box from the libhipspmv.so that had just passed the GPU tests ({note}); recorded "
                     f"{time.strftime('%Y-%m-%d %H:%M UTC', time.gmtime())}, tree commit {commit}."),
           "kernels": [{"validated": k, "current": k, "sha256": base[k]["sha256"], "insts": base[k]["insts"]}
                       for k in PRODUCT]}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"recorded {len(PRODUCT)} kernels -> {out}")


if __name__ == "__main__":
    main()
