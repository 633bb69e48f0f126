#!/usr/bin/env python3
"""k_vflow's per-wave cycle split on C3 (diagnostic): option
vflow_prof stamps every wave's waits; prints the means over the units of one
launch after --warm launches (loader: waiting for a free slot, issuing + waiting
for its DMA; compute: waiting for a panel, applying, issuing entry loads).
usage: vf_prof.py [--de 2,4] [--map 0]"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--de", default="2,4")
    p.add_argument("--map", type=int, default=0)
    p.add_argument("--warm", type=int, default=100)
    a = p.parse_args()
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32, 1, 2)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("vcache_flow")
    h.set_option("vflow_map", a.map)
    xd = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    yd = torch.empty(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    for de in (int(v) for v in a.de.split(",")):
        h.set_option("vflow_de", de)
        h.set_option("vflow_prof", 0)
        for _ in range(a.warm):
            h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
        h.set_option("vflow_prof", 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        h.exec_device(xd, yd, beta=0, mode=hs.MODE_FAST, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        keys = ["loader_freewait", "loader_dma", "loader_total", "compute_panelwait", "compute_apply",
                "compute_loads", "compute_total"]
        st = {k: h.stat("vflow_prof_" + k) for k in keys}
        print(f"de {de}: {e0.elapsed_time(e1) * 1e3:.1f} us (profiled launch); "
              + ", ".join(f"{k} {v}" for k, v in st.items()), flush=True)
    h.close()


if __name__ == "__main__":
    main()
