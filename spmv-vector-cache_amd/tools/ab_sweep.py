#!/usr/bin/env python3
"""A/B timing of FAST kernel configurations on C3 in the chip's steady state
(DESIGN.md §6.14).  Diagnostic only.

The first ~150 launches after an idle GPU run slower (a DVFS transient,
tools/warm_probe.py), so the sweep first runs 400 launches, then
times every configuration in interleaved rounds: per round and configuration,
10 untimed launches and N timed ones between one HIP event pair.  Each
configuration's result is checked once against the ORDERED kernel (bit-exact
to SoftwareSpMV, tests/test_gpu_parity.py) within the FAST bound, and for
determinism (two launches, identical bits).

usage: ab_sweep.py [--set NAME] [--reps N] [--rounds R]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402

SETS = {
    # round 5: the ORDERED loaders skipping the x lines no entry of a panel uses (option vcache_xmask)
    "xmask": [("ordered (product: xmask)", "vcache", {}), ("ordered xmask off", "vcache", {"vcache_xmask": 0}),
              ("ordered row order xmask", "bank0:vcache", {})],
    # round 5: ORDERED with 1/4 .. 3/4 of its row blocks' entries Infinity-Cache resident (256 blocks)
    "ordered_res": [("ordered (product: 1/2)", "vcache", {}), ("ordered resident 1/4", "vcache", {"vcache_nt": 64}),
                    ("ordered resident 3/8", "vcache", {"vcache_nt": 96}),
                    ("ordered resident 5/8", "vcache", {"vcache_nt": 160}),
                    ("ordered resident 3/4", "vcache", {"vcache_nt": 192}), ("ordered all nt", "vcache", {"vcache_nt": 0})],
    # round 5: ORDERED's first run continuation by DPP (xlane 6, the default on banked layouts) against
    # re-reading it from memory (xlane 0)
    "ordered6": [("ordered (product)", "vcache", {}), ("ordered xlane 0", "vcache", {"vcache_xlane": 0}),
                 ("ordered xlane 6", "vcache", {"vcache_xlane": 6}),
                 ("ordered LDS-DMA x", "vcache", {"vcache_dma": 1}),
                 ("ordered LDS-DMA x xlane 6", "vcache", {"vcache_dma": 1, "vcache_xlane": 6})],
    # round 5: k_vcache's four-part geometry (banked, LDS-DMA loaders, xlane 5, resident entries) against the
    # product; "v4:" a handle created with HIPSPMV_SPLIT4_VCACHE=1
    "split4": [("split (product)", "vcache_split", {}), ("vcache 4 parts", "v4:vcache_split4", {}),
               ("vcache 4 parts map 1", "v4:vcache_split4", {"vcache_map": 1}),
               ("vquad v0", "vcache_split4", {"vquad_variant": 0})],
    "resid2": [("split resident 1/2", "vcache_split", {"vcache_nt": 42}),
               ("split resident 7/16", "vcache_split", {"vcache_nt": 37}),
               ("split resident 17/32", "vcache_split", {"vcache_nt": 45}),
               ("split resident 9/16", "vcache_split", {"vcache_nt": 48}),
               ("split resident 1/2 map 2", "vcache_split", {"vcache_nt": 42, "vcache_map": 2}),
               ("split resident 9/16 map 2", "vcache_split", {"vcache_nt": 48, "vcache_map": 2}),
               ("split resident 5/8 map 2", "vcache_split", {"vcache_nt": 53, "vcache_map": 2})],
    # round 5: Infinity-Cache residency of the split kernel's entries on the banked layout (blocks < vcache_nt
    # load with the default policy; C3 has 85 row blocks)
    "resid": [("split all nt (product)", "vcache_split", {}),
              ("split resident 1/8", "vcache_split", {"vcache_nt": 11}),
              ("split resident 1/4", "vcache_split", {"vcache_nt": 21}),
              ("split resident 3/8", "vcache_split", {"vcache_nt": 32}),
              ("split resident 1/2", "vcache_split", {"vcache_nt": 42}),
              ("split resident 5/8", "vcache_split", {"vcache_nt": 53})],
    # round 5: the split kernel with one column part per XCD where it can (vcache_map 2)
    "map": [("split (product)", "vcache_split", {}), ("split map 2", "vcache_split", {"vcache_map": 2})],
    # round 5: the ORDERED vcache (bit-exact) on the banked layout, run continuation by memory re-reads
    # (xlane 0, the default), cross-lane (3) or DPP (5); checked bit-exact against the row-order layout
    "ordered": [("ordered banked xl0", "vcache", {}), ("ordered row order xl0", "bank0:vcache", {}),
                ("ordered banked xl3", "vcache", {"vcache_xlane": 3}),
                ("ordered banked xl5", "vcache", {"vcache_xlane": 5}),
                ("ordered banked xl5 nt none", "vcache", {"vcache_xlane": 5, "vcache_nt": 1 << 30}),
                ("ordered banked xl5 nt all", "vcache", {"vcache_xlane": 5, "vcache_nt": 0})],
    # round 5: the split kernel's first run-continuation step by DPP (xlane 5, the default on banked layouts)
    "dpp": [("split dpp (default)", "vcache_split", {}), ("split xlane 3", "vcache_split", {"vcache_xlane": 3}),
            ("split row order", "bank0:vcache_split", {})],
    # round 5: the split layout's LDS-bank-aware placement against the (row, column) order
    # ("bank0": a second handle created with HIPSPMV_VCACHE_BANK=0)
    "bank": [("split banked", "vcache_split", {}), ("split row order", "bank0:vcache_split", {}),
             ("vquad v0", "vcache_split4", {"vquad_variant": 0})],
    # round 5: k_vquad's XCD map, Infinity-Cache resident entries, LDS atomic y updates
    "vquad": [("split (product)", "vcache_split", {}),
              ("vquad v0", "vcache_split4", {"vquad_variant": 0}),
              ("vquad map", "vcache_split4", {"vquad_variant": 21}),
              ("vquad map res 1/4", "vcache_split4", {"vquad_variant": 22, "vcache_nt": 16}),
              ("vquad map res 3/8", "vcache_split4", {"vquad_variant": 22, "vcache_nt": 24}),
              ("vquad map res 1/2", "vcache_split4", {"vquad_variant": 22, "vcache_nt": 32}),
              ("vquad res 1/4", "vcache_split4", {"vquad_variant": 23, "vcache_nt": 16}),
              ("vquad res 1/2", "vcache_split4", {"vquad_variant": 23, "vcache_nt": 32}),
              ("vquad map yadd", "vcache_split4", {"vquad_variant": 24}),
              ("vquad map res 1/4 yadd", "vcache_split4", {"vquad_variant": 25, "vcache_nt": 16}),
              ("vquad yadd", "vcache_split4", {"vquad_variant": 26})],
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--set", default="vquad")
    p.add_argument("--reps", type=int, default=100)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32, 1, 2)
    x = hs.gen_vector(n, 3)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    hb = h4 = None
    if any(k.startswith("bank0:") for _, k, _ in SETS[a.set]):
        os.environ["HIPSPMV_VCACHE_BANK"] = "0"
        hb = hs.Handle.from_csr(rowptr, colind, vals, n, n)
        del os.environ["HIPSPMV_VCACHE_BANK"]
    if any(k.startswith("v4:") for _, k, _ in SETS[a.set]):
        os.environ["HIPSPMV_SPLIT4_VCACHE"] = "1"
        h4 = hs.Handle.from_csr(rowptr, colind, vals, n, n)
        h4.set_kernel("vcache_split4")  # the layout is built on first selection, while the variable is set
        del os.environ["HIPSPMV_SPLIT4_VCACHE"]
    alg = h.stat("alg_bytes")
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    # the reference: the ORDERED kernel (bit-exact to SoftwareSpMV by the GPU tests), on the row-order
    # layout when the set has that handle
    href = hb if hb is not None else h
    href.set_kernel("vcache")
    href.exec_device(xd, yd, beta=0, mode=hs.MODE_ORDERED, stream=s)
    y_ref = yd.cpu().numpy().copy()
    lens = np.diff(rowptr.astype(np.int64))
    absprod = np.bincount(np.repeat(np.arange(n), lens), weights=np.abs(vals * x[colind]), minlength=n)
    bound = 2.0 * lens * 2.0 ** -53 * absprod + 1e-300

    cfgs = SETS[a.set]

    cur = [h]

    def select(kernel, opts):
        cur[0] = hb if kernel.startswith("bank0:") else h4 if kernel.startswith("v4:") else h
        cur[0].set_kernel(kernel.split(":")[-1])
        for k, v in opts.items():
            cur[0].set_option(k, v)

    def reset(opts):
        for k in opts:
            cur[0].set_option(k, {"vquad_variant": 0, "vcache_nt": -1, "vcache_map": 0, "vcache_xmask": 1}.get(k, -1))

    mode = hs.MODE_ORDERED if a.set in ("ordered", "xmask", "ordered6", "ordered_res") else hs.MODE_FAST

    def run(k):
        for _ in range(k):
            cur[0].exec_device(xd, yd, beta=0, mode=mode, stream=s)

    checks = {}
    y_first = None
    for label, kernel, opts in cfgs:
        select(kernel, opts)
        run(1)
        y1 = yd.cpu().numpy().copy()
        run(1)
        y2 = yd.cpu().numpy().copy()
        r = np.abs(y1 - y_ref) / bound
        checks[label] = {"within_bound": bool(np.all(r <= 1.0)), "max_err_over_bound": round(float(r.max()), 3),
                         "deterministic": y1.tobytes() == y2.tobytes()}
        if mode == hs.MODE_ORDERED:  # y_ref came from the ordered kernel on the row-order layout? (below)
            checks[label]["bit_exact_vs_ordered_ref"] = y1.tobytes() == y_ref.tobytes()
        if y_first is None:
            y_first = y1
        else:
            checks[label]["bits_equal_first_config"] = y1.tobytes() == y_first.tobytes()
        reset(opts)
    select(cfgs[0][1], cfgs[0][2])
    run(400)
    reset(cfgs[0][2])
    torch.cuda.synchronize()
    times = {c[0]: [] for c in cfgs}
    for rnd in range(a.rounds):
        for label, kernel, opts in cfgs:
            select(kernel, opts)
            run(10)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            run(a.reps)
            e1.record(s)
            torch.cuda.synchronize()
            times[label].append(e0.elapsed_time(e1) * 1e3 / a.reps)
            reset(opts)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    for label, _, _ in cfgs:
        us = float(np.median(times[label]))
        print(f"{label:28s} {us:8.2f} us  frac {alg / (us * 1e-6) / 8e12:.4f}  "
              f"rounds {' '.join(f'{t:.1f}' for t in times[label])}  {json.dumps(checks[label])}", flush=True)
    h.close()


if __name__ == "__main__":
    main()
