#!/usr/bin/env python3
"""A/B of option settings on C5 shards (R-MAT scale 24 cut by the library's
partition, hipspmv_partition_rows), each shard timed alone on this GPU in the
chip's steady state; results must keep their bits.  Diagnostic only
(DESIGN.md §6.15).

usage: c5_ab.py [--shards 0,3,7] [--set NAME] [--rounds R]
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402

# settings: (label, {option: value or ("groups", fraction)})
SETS = {
    "one": [("product", {})],
    "fill": [("fill beside the segment pass", {"wcsr_fill": 1}), ("fill after the reduce", {"wcsr_fill": 0})],
    "reduce": [("compact reduce", {}), ("all-rows reduce", {"wcsr_reduce": 1})],
    "xcd": [("product", {}), ("xcd eighths", {"wcsr_xcd": 1})],
    "wg": [("product", {}), ("wgather (kernel 6)", {"kernel": 6})],
    "res": [("all nt (product)", {}), ("resident 1/8", {"wcsr_res": ("groups", 0.125)}),
            ("resident 1/4", {"wcsr_res": ("groups", 0.25)}), ("resident 3/8", {"wcsr_res": ("groups", 0.375)}),
            ("resident 1/2", {"wcsr_res": ("groups", 0.5)})],
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shards", default="0,3,7")
    p.add_argument("--set", default="res")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=30)
    p.add_argument("--scale", type=int, default=24)
    a = p.parse_args()
    n = 1 << a.scale
    rowptr, colind, vals = hs.gen_rmat_csr(a.scale)
    bounds = hs.partition_rows_cost(rowptr, colind, n, 8)
    x = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    s = torch.cuda.current_stream()
    cfgs = SETS[a.set]
    for sh in (int(v) for v in a.shards.split(",")):
        r0, r1 = int(bounds[sh]), int(bounds[sh + 1])
        e0, e1 = int(rowptr[r0]), int(rowptr[r1])
        rp = (rowptr[r0:r1 + 1].astype(np.int64) - e0).astype(np.uint32)
        h = hs.Handle.from_csr(rp, colind[e0:e1], vals[e0:e1], r1 - r0, n)
        y = torch.empty(r1 - r0, dtype=torch.float64, device="cuda")
        groups = h.stat("wcsr_groups") if h.kernel_name(hs.MODE_FAST) == "wcsr" else 0

        def opts(o):
            for k, v in o.items():
                h.set_option(k, int(groups * v[1]) if isinstance(v, tuple) else v)

        def reset(o):
            for k in o:
                h.set_option(k, {"wcsr_fill": -1}.get(k, 0))

        def run(k):
            for _ in range(k):
                h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=s)

        run(200)
        torch.cuda.synchronize()
        y0 = y.cpu().numpy().copy()
        times = {c[0]: [] for c in cfgs}
        same = {}
        for _ in range(a.rounds):
            for label, o in cfgs:
                opts(o)
                run(10)
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record(s)
                run(a.reps)
                ev1.record(s)
                torch.cuda.synchronize()
                times[label].append(ev0.elapsed_time(ev1) * 1e3 / a.reps)
                same[label] = y.cpu().numpy().tobytes() == y0.tobytes()
                reset(o)
        alg = h.stat("alg_bytes")
        for label, _ in cfgs:
            us = float(np.median(times[label]))
            print(f"shard {sh} ({h.kernel_name(hs.MODE_FAST)}, {groups} groups)  {label:22s} {us:8.2f} us  "
                  f"frac {alg / (us * 1e-6) / 8e12:.4f}  same bits {same[label]}  "
                  f"rounds {' '.join(f'{t:.1f}' for t in times[label])}", flush=True)
        h.close()


if __name__ == "__main__":
    main()
