#!/usr/bin/env python3
"""ORDERED k_sell on a C5 shard: the product (hub rows of >= kSellIso entries
as isolated chains, k_sell_iso<kIsoG>) against the forms of option
"sell_chain" (needs HIPSPMV_EXPERIMENTAL=1): 1 no isolated chains (k_sell),
2 / 3 isolated chains with G = 12 (12 helper waves) / 30 products per lane
per stage.
Every form adds the same products in the same order, so the bits must match
the product's.  Then the hub rows alone, the longest row alone and the slices
alone (timing only).  Not part of the product.

    HIPSPMV_EXPERIMENTAL=1 python tools/chain_sweep.py [--shard 0]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipspmv as hs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--scale", type=int, default=24)
p.add_argument("--shard", type=int, default=0)
p.add_argument("--reps", type=int, default=10)
a = p.parse_args()
bounds = hs.partition_row_counts(hs.gen_rmat_row_counts(a.scale, 16, 4), 8)
r0, r1 = int(bounds[a.shard]), int(bounds[a.shard + 1])
rowptr, colind, vals = hs.gen_rmat_rows(a.scale, r0, r1, 16, 4)
rows, cols = r1 - r0, 1 << a.scale
x = torch.from_numpy(hs.gen_vector(cols, 3)).cuda()
y = torch.empty(rows, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
alg = 12 * colind.size + 4 * (rows + 1) + 8 * cols + 8 * rows
h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
h.set_kernel("sell")
ref = None
for rnd in range(1):
    for g in (0, 1, 2, 3):
        h.set_option("sell_chain", g)
        for _ in range(2):
            h.exec_device(x, y, beta=0, mode=hs.MODE_ORDERED, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            h.exec_device(x, y, beta=0, mode=hs.MODE_ORDERED, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        yy = y.cpu().numpy().copy()
        ref = yy if ref is None else ref
        same = yy.tobytes() == ref.tobytes()
        print(f"round {rnd} shard {a.shard} chain {('product (isolated G=45)', 'not isolated (k_sell)', 'isolated G=12 (12 helper waves)', 'isolated G=30')[g]}: {us:8.1f} us  frac8TB={alg / us / 1e3 / 8000:.4f}"
              f"  {'bit-identical to product' if same else 'BITS DIFFER'}", flush=True)
# where the time goes: the hub chains alone, the slices alone (timing only)
for only, label in ((1, "hub rows only"), (3, "longest row only"), (2, "slices only")):
    for g in ((0, 2) if only != 2 else (0,)):
        h.set_option("sell_chain", g)
        h.set_option("sell_only", only)
        for _ in range(2):
            h.exec_device(x, y, beta=0, mode=hs.MODE_ORDERED, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            h.exec_device(x, y, beta=0, mode=hs.MODE_ORDERED, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        print(f"{label:14s} chain {g or 'product'}: {e0.elapsed_time(e1) / a.reps * 1e3:8.1f} us", flush=True)
    h.set_option("sell_only", 0)
lens = np.diff(rowptr.astype(np.int64))
top = np.sort(lens)[::-1][:12]
print("isolated hub rows:", h.stat("sell_iso_hubs"), "longest rows:", top.tolist(), "rows > 256:", int(np.sum(lens > 256)), "rows > 32768:", int(np.sum(lens > 32768)))
h.close()
