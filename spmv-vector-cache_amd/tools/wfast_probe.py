#!/usr/bin/env python3
"""Design probe for a windowed FAST path on C5 shards.

C5 shard 0 of 8 (R-MAT scale 24, rows [0, 70272), 31.7 M nnz) gathers x from
all 16 M columns; its x traffic is ~4x the algorithmic bytes although only
664 k distinct 128-B lines of x are touched.  Cutting every row at column
windows gives a "segment matrix" A' (one virtual row per (window, row) pair,
in window-major order): a kernel that walks A' in order gathers from one
window at a time, and y is the per-row sum of the segment partials.

This probe times the existing kernels on A' against A (kernel time only, the
per-row reduce is not included) to decide whether the path is worth
building.  Not part of the product.

    python tools/wfast_probe.py [--log2-window 19] [--shard 0]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hipspmv as hs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--scale", type=int, default=24)
p.add_argument("--shard", type=int, default=0)
p.add_argument("--windows", default="17,19,21")
p.add_argument("--c4", action="store_true", help="C4 shard (stripe 2^21 x 2^24, 32 nnz/row) instead of R-MAT")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--only-wcsr", action="store_true", help="time the wcsr kernel only")
a = p.parse_args()

t0 = time.time()
if a.c4:
    rows, cols = 1 << 21, 1 << a.scale
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32)
else:
    bounds = hs.partition_row_counts(hs.gen_rmat_row_counts(a.scale, 16, 4), 8)
    r0, r1 = int(bounds[a.shard]), int(bounds[a.shard + 1])
    rowptr, colind, vals = hs.gen_rmat_rows(a.scale, r0, r1, 16, 4)
    rows, cols = r1 - r0, 1 << a.scale
print(f"shard {a.shard}: rows {rows} nnz {colind.size} (gen {time.time() - t0:.1f} s)", flush=True)
x = torch.from_numpy(hs.gen_vector(cols, 3)).cuda()
s = torch.cuda.current_stream()


def timeit(h, mode, yd):
    for _ in range(3):
        h.exec_device(x, yd, beta=0, mode=mode, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        h.exec_device(x, yd, beta=0, mode=mode, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps * 1e3


alg = 12 * colind.size + 4 * (rows + 1) + 8 * cols + 8 * rows
h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
y = torch.empty(rows, dtype=torch.float64, device="cuda")
for k in (("wcsr",) if a.only_wcsr else ("sell", "csr_vector", "wgather", "wcsr")):
    try:
        h.set_kernel(k)
    except hs.HipSpMVError:
        continue
    us = timeit(h, hs.MODE_FAST, y)
    extra = (f" (window 2^{h.stat('wcsr_window_log2')}, {h.stat('wcsr_segments')} segments, "
             f"{h.stat('wcsr_chunks')} LDS chunks)") if k == "wcsr" else ""
    print(f"A  {k:10s} FAST {us:8.1f} us  frac8TB={alg / us / 1e3 / 8000:.3f}{extra}", flush=True)
h.close()

lens = np.diff(rowptr.astype(np.int64))
row_of = np.repeat(np.arange(rows, dtype=np.int64), lens)
for lw in [int(v) for v in a.windows.split(",") if v]:
    win = colind.astype(np.int64) >> lw
    key = win * rows + row_of  # window-major, then row; each row's entries stay in column order
    order = np.argsort(key, kind="stable")
    k_sorted = key[order]
    seg_start = np.flatnonzero(np.r_[True, k_sorted[1:] != k_sorted[:-1]])
    nseg = seg_start.size
    rp2 = np.r_[seg_start, k_sorted.size].astype(np.uint32)
    c2 = colind[order]
    v2 = vals[order]
    l2 = np.diff(rp2.astype(np.int64))
    print(f"W=2^{lw}: {nseg} segments, longest {l2.max()}", flush=True)
    h2 = hs.Handle.from_csr(rp2, c2, v2, nseg, cols)
    y2 = torch.empty(nseg, dtype=torch.float64, device="cuda")
    for k in ("csr_vector",):
        h2.set_kernel(k)
        us = timeit(h2, hs.MODE_FAST, y2)
        print(f"A' {k:10s} FAST {us:8.1f} us  frac8TB={alg / us / 1e3 / 8000:.3f} (segment partials only)",
              flush=True)
    h2.close()
