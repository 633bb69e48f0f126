#!/usr/bin/env python3
"""The NewCache state statistics (option "profile") of the
vcache kernels on the C3 matrix: where a launch's time goes per workgroup.

    python tools/profile_states.py [--log2-rows 20] [--log2-cols 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipspmv as hs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--log2-rows", type=int, default=20)
p.add_argument("--log2-cols", type=int, default=20)
a = p.parse_args()
rows, cols = 1 << a.log2_rows, 1 << a.log2_cols
rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
x = hs.gen_vector(cols, 3)
h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
keys = ["fill", "active", "flush", "done", "read_miss2"]
for kernel, mode in [("vcache_split", hs.MODE_FAST), ("vcache", hs.MODE_ORDERED)]:
    h.set_kernel(kernel)
    h.set_option("profile", 1)
    for _ in range(5):
        h.exec(x, beta=0, mode=mode)
    ghz = h.stat("clock_khz") / 1e6
    us = {k: h.stat("state_" + k) / ghz / 1e3 for k in keys}
    us["no_valid_but_ready"] = h.stat("no_valid_but_ready") / ghz / 1e3
    us["no_ready_but_valid"] = h.stat("no_ready_but_valid") / ghz / 1e3
    span = h.stat("profile_span_cycles") / ghz / 1e3
    print(f"{kernel:13s} span {span:7.2f} us (kernel {h.stat('kernel_ns') / 1e3:7.2f} us, "
          f"{h.stat('profile_units')} workgroups) -- means per workgroup, us: "
          + ", ".join(f"{k} {v:.2f}" for k, v in us.items()), flush=True)
    h.set_option("profile", 0)
h.close()
