#!/usr/bin/env python3
"""A/B of the wide-x FAST kernels on C4 shards (diagnostic):
k_wgather (one part, 8192-row blocks on a 2^21-row shard) against
k_wgather_split (two column halves of 16384-row blocks, part 0 on XCDs 0-3,
part 1 on XCDs 4-7).  Shards of the 2^24 x 2^24 stripe matrix (32 nnz/row),
each created alone as the 8-GPU job creates them; interleaved rounds of
--launches back-to-back launches after --warm launches, HIP events on the
launch stream.  Prints per (shard, kernel) the median and best round (us per
launch) and the fraction of 8 TB/s (algorithmic bytes), and checks that the
two kernels agree within twice the FAST bound and that each is deterministic.
usage: wgs_ab.py [--shards 0,7] [--rounds R] [--launches N] [--warm W]"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shards", default="0,7")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=50)
    p.add_argument("--warm", type=int, default=100)
    p.add_argument("--kernels", default="wgather,wgather_split")
    p.add_argument("--parts", type=int, default=8, help="shards of the C4 matrix (rows = 2^24 / parts)")
    p.add_argument("--nt", default="", help="wgather_split entry residency sweep: vcache_nt values (first "
                   "non-temporal block), e.g. 0,16,32")
    a = p.parse_args()
    n = 1 << 24
    rows = n // a.parts
    x = hs.gen_vector(n, 3)
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty(rows, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    kernels = a.kernels.split(",")
    if a.nt:  # configurations "wgather_split@K": option vcache_nt = K
        kernels = [k for k in kernels if k != "wgather_split"] + [f"wgather_split@{v}" for v in a.nt.split(",")]
    for shard in (int(v) for v in a.shards.split(",")):
        rp, ci, va = hs.gen_stripe_csr(shard * rows, rows, n, 32)
        h = hs.Handle.from_csr(rp, ci, va, rows, n)
        print(f"shard {shard}: AUTO FAST {h.kernel_name(hs.MODE_FAST)}, setup {h.stat('setup_ns') / 1e9:.2f} s, "
              f"split rows/block {h.stat('wgather_split_rows_per_block')}", flush=True)
        def select(k):  # "kernel", "kernel@NT" (option vcache_nt), "wgather_split#alt" (option wgather_map 1)
            name, _, alt = k.partition("#")
            name, _, nt = name.partition("@")
            h.set_kernel(name)
            h.set_option("vcache_nt", int(nt) if nt else -1)
            if name == "wgather_split":
                h.set_option("wgather_map", 1 if alt == "alt" else 0)

        for k in kernels:  # build both layouts before timing
            select(k)
        absprod = np.bincount(np.repeat(np.arange(rows), 32), weights=np.abs(va * x[ci]), minlength=rows)
        bound = 2.0 * 33 * 2.0 ** -53 * absprod + 1e-300
        del rp, ci
        times = {k: [] for k in kernels}
        bits, res = {}, {}
        for r in range(a.rounds):
            for k in kernels:
                select(k)
                for _ in range(a.warm if r == 0 else 10):
                    h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.launches):
                    h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / a.launches)
                res[k] = h.stat("resident_entry_bytes")
                y = yd.cpu().numpy().tobytes()
                assert bits.setdefault(k, y) == y, f"{k}: bits changed between launches"
                print(f"  round {r} {k}: {times[k][-1]:.1f} us", flush=True)
        alg = h.stat("alg_bytes")
        ys = {k: np.frombuffer(bits[k], dtype=np.float64) for k in kernels}
        for k in kernels:
            t = np.array(times[k])
            msg = ""
            if len(kernels) > 1:
                dev = float(np.max(np.abs(ys[k] - ys[kernels[0]]) / bound))
                assert dev <= 2.0, (k, dev)
                msg = f", |y - y_{kernels[0]}| / bound max {dev:.3f}"
            print(f"shard {shard} {k}: resident {res[k] / 1e6:.0f} MB, median {np.median(t):.1f} us, best {t.min():.1f} us, "
                  f"frac {alg / (np.median(t) * 1e-6) / 8e12:.4f}{msg}", flush=True)
        h.close()


if __name__ == "__main__":
    main()
