#!/usr/bin/env python3
"""Time every applicable kernel on one synthetic matrix (HIP events, back-to-back
launches on one stream) -- the A/B table behind DESIGN.md's kernel choices."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipspmv as hs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--log2-rows", type=int, default=20)
p.add_argument("--log2-cols", type=int, default=20)
p.add_argument("--k", type=int, default=32)
p.add_argument("--rmat", type=int, default=0, help="R-MAT scale instead of the stripe generator")
p.add_argument("--reps", type=int, default=50)
p.add_argument("--rounds", type=int, default=3)
a = p.parse_args()
if a.rmat:
    rowptr, colind, vals = hs.gen_rmat_csr(a.rmat, 16, 4)
    rows = cols = 1 << a.rmat
    name = f"rmat{a.rmat}"
else:
    rows, cols = 1 << a.log2_rows, 1 << a.log2_cols
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, a.k)
    name = f"stripe {rows}x{cols} k={a.k}"
h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
x = torch.from_numpy(hs.gen_vector(cols, 3)).cuda()
y = torch.empty(rows, dtype=torch.float64, device="cuda")
alg = h.stat("alg_bytes")
s = torch.cuda.current_stream()
cands = [("vcache", hs.MODE_ORDERED), ("csr_lane", hs.MODE_ORDERED), ("vcache_split", hs.MODE_FAST),
         ("csr_vector", hs.MODE_FAST)]
res = {}
for rnd in range(a.rounds):  # interleaved rounds in one process (methodology rule 24)
    for kname, mode in cands:
        try:
            h.set_kernel(kname)
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        except hs.HipSpMVError:
            continue
        for _ in range(3):
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        res.setdefault(kname, []).append(e0.elapsed_time(e1) / a.reps * 1e3)
print(f"{name}: nnz={colind.size} alg_bytes={alg}")
for kname, ts in res.items():
    us = float(np.median(ts))
    print(f"  {kname:14s} {us:9.2f} us  {alg / us / 1e3:8.1f} GB/s  {2 * colind.size / us / 1e3:8.1f} GFLOP/s"
          f"  frac8TB={alg / us / 1e3 / 8000:.3f}  (rounds: {', '.join(f'{t:.1f}' for t in ts)})")
