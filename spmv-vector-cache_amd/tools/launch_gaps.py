#!/usr/bin/env python3
"""Gaps between back-to-back eager launches of the C3 FAST kernel (diagnostic,
DESIGN.md §7): run under `rocprofv3 --kernel-trace`; prints the kernel
durations and the idle time between consecutive dispatches of the timed
launches, after a warm-up.  usage: launch_gaps.py [--launches N]"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=40)
    a = p.parse_args()
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32, 1, 2)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    xd = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    yd = torch.empty(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(300):
        h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.launches):
        h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{a.launches} eager launches: {e0.elapsed_time(e1) * 1e3 / a.launches:.2f} us per launch (events)", flush=True)
    h.close()


if __name__ == "__main__":
    main()
