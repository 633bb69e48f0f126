#!/usr/bin/env python3
"""ORDERED k_sell on a C5 shard: the product hub chain (kChainG entries per
lane per stage) against the experimental forms of option "sell_chain" (10 * G + D: G entries per lane
per stage, gathers D stages ahead)
(needs HIPSPMV_EXPERIMENTAL=1).  Every form adds the same products in the
same order, so the bits must match the product's.  Not part of the product.

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
for rnd in range(2):
    for g in (0, 82, 121, 122, 161):
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
        print(f"round {rnd} shard {a.shard} chain {'G=%d D=%d' % (g // 10, g % 10) if g else 'product G=8 D=1'}: {us:8.1f} us  frac8TB={alg / us / 1e3 / 8000:.4f}"
              f"  {'bit-identical to product' if same else 'BITS DIFFER'}", flush=True)
h.close()
