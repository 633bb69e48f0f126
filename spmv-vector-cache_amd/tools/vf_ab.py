#!/usr/bin/env python3
"""A/B of the C3 FAST kernels in the steady state (diagnostic):
vcache_split (product) against k_vflow configurations, interleaved rounds of
--launches back-to-back launches after --warm launches each, HIP events on the
launch stream.  Prints per configuration the median and best round (us per
launch), and checks that every configuration's bits are stable across launches
and that each stays within twice the FAST bound of vcache_split's result
(both are within the bound of the exact sums).
usage: vf_ab.py [--rounds R] [--launches N] [--warm W] [--configs a,b,...]"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402

CONFIGS = {
    "split": ("vcache_split", {}),
    "flow": ("vcache_flow", {"vflow_map": 0}),
    "flow_map1": ("vcache_flow", {"vflow_map": 1}),
    "flow_allnt": ("vcache_flow", {"vflow_map": 0, "vcache_nt": 0}),
    "flow_map1_allnt": ("vcache_flow", {"vflow_map": 1, "vcache_nt": 0}),
    "split_allnt": ("vcache_split", {"vcache_nt": 0}),
    "flow_res58": ("vcache_flow", {"vflow_map": 0, "vcache_nt": 40}),
    "flow_res38": ("vcache_flow", {"vflow_map": 0, "vcache_nt": 24}),
    "flow_de2": ("vcache_flow", {"vflow_map": 0, "vflow_de": 2}),
    "flow_de3": ("vcache_flow", {"vflow_map": 0, "vflow_de": 3}),
    "flow_de4": ("vcache_flow", {"vflow_map": 0, "vflow_de": 4}),
    "flow_de8": ("vcache_flow", {"vflow_map": 0, "vflow_de": 8}),
    "flow_map1_de3": ("vcache_flow", {"vflow_map": 1, "vflow_de": 3}),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--launches", type=int, default=100)
    p.add_argument("--warm", type=int, default=300)
    p.add_argument("--configs", default="split,flow,flow_map1")
    a = p.parse_args()
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32, 1, 2)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("vcache_flow")  # build its layout once (the handle keeps both)
    print(f"vflow layout: units {h.stat('vflow_units')}, max group {h.stat('vflow_max_group')}", flush=True)
    xd = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    yd = torch.empty(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    absprod = np.zeros(n)
    np.add.at(absprod, np.repeat(np.arange(n), 32), np.abs(vals * hs.gen_vector(n, 3)[colind]))
    bound = 2.0 * 32 * 2.0 ** -53 * absprod + 1e-300
    names = a.configs.split(",")

    def setup(name):
        kern, opts = CONFIGS[name]
        h.set_kernel(kern)
        h.set_option("vcache_nt", -1)
        if kern == "vcache_flow":
            h.set_option("vflow_map", 0)
            h.set_option("vflow_de", 4)
        for k, v in opts.items():
            h.set_option(k, v)

    ref = None
    times = {k: [] for k in names}
    bits = {}
    for r in range(a.rounds):
        for name in names:
            setup(name)
            for _ in range(a.warm if r == 0 else 20):
                h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.launches):
                h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
            e1.record(s)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / a.launches)
            y = yd.cpu().numpy().copy()
            if name in bits:
                assert y.tobytes() == bits[name], f"{name}: bits changed between launches"
            bits[name] = y.tobytes()
            if name == "split":
                ref = y
            print(f"round {r} {name}: {times[name][-1]:.2f} us", flush=True)
    alg = h.stat("alg_bytes")
    for name in names:
        t = np.array(times[name])
        msg = ""
        if ref is not None:
            y = np.frombuffer(bits[name], dtype=np.float64)
            msg = f", |y - y_split| / bound max {float(np.max(np.abs(y - ref) / bound)):.3f}"
        print(f"{name}: median {np.median(t):.2f} us, best {t.min():.2f} us, frac {alg / (np.median(t) * 1e-6) / 8e12:.4f}"
              f"{msg}", flush=True)
    if "vcache_flow" in [CONFIGS[k][0] for k in names]:
        print("vflow_timeouts", h.stat("vflow_timeouts"), flush=True)
    h.close()


if __name__ == "__main__":
    main()
