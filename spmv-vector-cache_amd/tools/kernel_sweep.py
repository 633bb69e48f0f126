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
p.add_argument("--only", default="", help="comma-separated label substrings to keep")
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
O, F = hs.MODE_ORDERED, hs.MODE_FAST
# (label, kernel, mode, options); the experimental ones need HIPSPMV_EXPERIMENTAL=1 at create
cands = [("vcache", "vcache", O, {}), ("csr_lane", "csr_lane", O, {}), ("vcache_split", "vcache_split", F, {}),
         ("csr_vector", "csr_vector", F, {}), ("sell", "sell", O, {}), ("sell fast", "sell", F, {}),
         ("wgather", "wgather", O, {}), ("wgather c128", "wgather", O, {"wgather_chunk": 128}),
         ("wgather c512", "wgather", O, {"wgather_chunk": 512}), ("wgather c0", "wgather", O, {"wgather_chunk": 0}),
         ("wgather c192", "wgather", O, {"wgather_chunk": 192}), ("wgather c320", "wgather", O, {"wgather_chunk": 320}),
         ("wgather c384", "wgather", O, {"wgather_chunk": 384}),
         ("wgather xl2", "wgather", O, {"vcache_xlane": 2}),
         # non-temporal entry loads from a fraction of the row blocks / slices on
         ("vcache nt all", "vcache", O, {"vcache_nt": 0}), ("vcache nt none", "vcache", O, {"vcache_nt": 1 << 30}),
         ("vcache nt 1/2", "vcache", O, {"vcache_nt": ("vcache_blocks", 0.5)}),
         ("vcache nt 1/4", "vcache", O, {"vcache_nt": ("vcache_blocks", 0.25)}),
         ("split nt none", "vcache_split", F, {"vcache_nt": 1 << 30}),
         ("split nt 1/4", "vcache_split", F, {"vcache_nt": ("vcache_split_units", 0.25 / 3)}),
         ("sell nt none", "sell", O, {"sell_nt": 1 << 30}),
         ("sell nt 3/8", "sell", O, {"sell_nt": ("sell_slices", 0.375)}),
         ("sell nt 1/2", "sell", O, {"sell_nt": ("sell_slices", 0.5)}),
         ("sell nt 5/8", "sell", O, {"sell_nt": ("sell_slices", 0.625)}),
         ("sell fast nt 1/2", "sell", F, {"sell_nt": ("sell_slices", 0.5)}),
         ("wcsr", "wcsr", F, {}),
         ("wgather nt", "wgather", O, {"vcache_nt": 0}), ("wgather no nt", "wgather", O, {"vcache_nt": 1 << 30})]
if os.environ.get("HIPSPMV_EXPERIMENTAL") == "1":
    cands += [("vcache xl1", "vcache", O, {"vcache_xlane": 1}), ("vcache xl2", "vcache", O, {"vcache_xlane": 2}),
              ("vcache dma", "vcache", O, {"vcache_dma": 1}),
              ("vcache dma xl2", "vcache", O, {"vcache_dma": 1, "vcache_xlane": 2}),
              ("split xl1", "vcache_split", F, {"vcache_xlane": 1}), ("split xl2", "vcache_split", F, {"vcache_xlane": 2}),
              ("split dma", "vcache_split", F, {"vcache_dma": 1}),
              ("split dma xl2", "vcache_split", F, {"vcache_dma": 1, "vcache_xlane": 2}),
              ("vcache xl3", "vcache", O, {"vcache_xlane": 3}), ("split xl3", "vcache_split", F, {"vcache_xlane": 3}),
              ("split4", "vcache_split4", F, {}), ("split4 xl2", "vcache_split4", F, {"vcache_xlane": 2}),
              ("split4 dma xl2", "vcache_split4", F, {"vcache_dma": 1, "vcache_xlane": 2}),
              ("split4 xl3", "vcache_split4", F, {"vcache_xlane": 3}),
              ("split4 dma xl3", "vcache_split4", F, {"vcache_dma": 1, "vcache_xlane": 3}),
              ("split4 map", "vcache_split4", F, {"vcache_map": 1}),
              ("split4 map xl3", "vcache_split4", F, {"vcache_map": 1, "vcache_xlane": 3}),
              ("split4 map xl2", "vcache_split4", F, {"vcache_map": 1, "vcache_xlane": 2}),
              ("split4 nt", "vcache_split4", F, {"vcache_nt": 0}),
              ("split4 dma xl3 nt", "vcache_split4", F, {"vcache_dma": 1, "vcache_xlane": 3, "vcache_nt": 0}),
              ("split4 map xl3 nt", "vcache_split4", F, {"vcache_map": 1, "vcache_xlane": 3, "vcache_nt": 0})]
if a.only:
    keep = a.only.split(",")
    # "=label" keeps that label only; anything else keeps the labels containing it
    cands = [c for c in cands
             if any((c[0] == k[1:]) if k.startswith("=") else (k in c[0]) for k in keep) or c[0] == "vcache"]
ref = None
res, check = {}, {}
for rnd in range(a.rounds):  # interleaved rounds in one process (methodology rule 24)
    for label, kname, mode, opts in cands:
        try:
            h.set_kernel(kname)
            for k in ("vcache_dma", "vcache_xlane", "vcache_map", "wgather_chunk", "vcache_nt", "sell_nt"):
                v = opts.get(k, {"vcache_xlane": -1, "vcache_dma": -1, "wgather_chunk": 256, "vcache_nt": -1,
                                 "sell_nt": -1}.get(k, 0))
                if isinstance(v, tuple):  # (statistic, fraction): a threshold relative to the layout
                    v = int(h.stat(v[0]) * v[1])
                h.set_option(k, v)
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        except hs.HipSpMVError:
            continue
        if rnd == 0:  # correctness vs the first ordered result: bits (ordered) or relative size (fast)
            torch.cuda.synchronize()
            yy = y.cpu().numpy().copy()
            if ref is None and mode == O:
                ref = yy
            if ref is not None:
                check[label] = ("bit-exact" if yy.tobytes() == ref.tobytes() else
                                f"max|d|={float(np.max(np.abs(yy - ref))):.2e}")
        for _ in range(3):
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            h.exec_device(x, y, beta=0, mode=mode, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        res.setdefault(label, []).append(e0.elapsed_time(e1) / a.reps * 1e3)
print(f"{name}: nnz={colind.size} alg_bytes={alg}")
for label, ts in res.items():
    us = float(np.median(ts))
    print(f"  {label:16s} {us:9.2f} us  {alg / us / 1e3:8.1f} GB/s  {2 * colind.size / us / 1e3:8.1f} GFLOP/s"
          f"  frac8TB={alg / us / 1e3 / 8000:.3f}  {check.get(label, '')}  (rounds: {', '.join(f'{t:.1f}' for t in ts)})")
