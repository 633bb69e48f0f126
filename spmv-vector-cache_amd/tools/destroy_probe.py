#!/usr/bin/env python3
"""What destroying a handle costs a launch loop on another handle (diagnostic,
DESIGN.md §9.5).

A 2^18 x 2^24 stripe handle (AUTO: wgather) runs --launches back-to-back launches timed by one
event pair, as tests/test_gpu_multi.py times its shards; a second, large handle
(2^22 rows of the C4 stripe matrix, several GB on the device, like the handles
earlier tests leave to the garbage collector) is destroyed after
launch --at, inside the timed region.  Reported: the per-launch time of the loop
with and without the destroy, and the host time of the destroy call.  Run it
once with HIPSPMV_SYNC_RELEASE=1 (the round-5 synchronous hipFree on the
caller's thread) and once without (the release thread); under rocprofv3
--kernel-trace the gap between the two launches around the destroy is visible
directly.  usage: destroy_probe.py [--launches N] [--at K]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--at", type=int, default=5)
    a = p.parse_args()
    mode = "synchronous hipFree (HIPSPMV_SYNC_RELEASE=1)" if os.environ.get("HIPSPMV_SYNC_RELEASE") == "1" \
        else "release thread"
    n = 1 << 24
    rp, ci, v = hs.gen_stripe_csr(0, 1 << 18, n, 32, 1, 2)  # the timed handle: 2^18 x 2^24 (AUTO: wgather)
    h = hs.Handle.from_csr(rp, ci, v, 1 << 18, n)
    x = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    y = torch.empty(1 << 18, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(30):
        h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=s)
    torch.cuda.synchronize()
    ref = y.cpu().numpy().copy()

    def loop(victim):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dt = None
        e0.record(s)
        for i in range(a.launches):
            h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=s)
            if victim is not None and i == a.at:
                t0 = time.perf_counter()
                victim.close()  # hipspmv_destroy
                dt = (time.perf_counter() - t0) * 1e3
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.launches, dt

    base, _ = loop(None)
    rb, cb, vb = hs.gen_stripe_csr(1 << 21, 1 << 22, n, 32, 1, 2)
    big = hs.Handle.from_csr(rb, cb, vb, 1 << 22, n)
    del rb, cb, vb
    dev_gb = big.stat("device_bytes") / 1e9
    xb = torch.empty(n, dtype=torch.float64, device="cuda")
    yb = torch.empty(1 << 22, dtype=torch.float64, device="cuda")
    big.exec_device(xb, yb, beta=0, mode=hs.MODE_FAST, stream=s)
    torch.cuda.synchronize()
    with_destroy, dt = loop(big)
    hs.release_wait()
    assert y.cpu().numpy().tobytes() == ref.tobytes()
    print(f"{mode}: {a.launches} launches {base:.1f} us each without a destroy, {with_destroy:.1f} us each with "
          f"a {dev_gb:.1f} GB handle destroyed after launch {a.at} (destroy call {dt:.2f} ms on the host)", flush=True)
    h.close()


if __name__ == "__main__":
    main()
