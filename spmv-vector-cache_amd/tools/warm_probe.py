"""Why a 20-launch C3 run measures slower per launch than a 200-launch one
(DESIGN.md §7).  Diagnostic only, not part of the bench.

Runs the headline handle (C3 FAST, vcache_split) through phases that differ
only in what the GPU did just before them, timing each launch with a HIP event
pair on the launch stream, and reads the effective shader clock of single
profiled launches (option "profile": loader wave 0's s_memtime cycles over the
main loop's s_memrealtime span, csrc/vcache.hip AB bit 128).  Run it under
`rocprofv3 --kernel-trace` as well to get the dispatch durations without
events (tools/warm_trace.py splits that trace into the same phases).

Phases (in this order, every one on the same handle and buffers):
  A  bench-like: 5 warmup launches, sync, 20 launches (one event pair)
  B  the same 20 launches with an event pair around each
  C  1 s idle, then 20 launches (pair)
  D  300 back-to-back launches (pair), then at once 20 more (pair)
  E  1 s idle, 0.5 s of a HBM copy loop, then 20 launches (pair)
  F  1 s idle, 0.5 s of back-to-back SpMV launches, 20 launches (pair)
  G  profiled single launches: after 1 s idle; after 300 launches
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hipspmv as hs  # noqa: E402


def main():
    rows = cols = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 32, 1, 2)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols, device=0)
    xd = torch.from_numpy(hs.gen_vector(cols)).cuda()
    yd = torch.empty(rows, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    mode = hs.MODE_FAST
    out = {"kernel": h.kernel_name(mode)}

    def launch(n):
        for _ in range(n):
            h.exec_device(xd, yd, beta=0, mode=mode, stream=s)

    def pair(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch(n)
        e1.record(s)
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / n, 2)

    def each(n):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        evs[0].record(s)
        for i in range(n):
            launch(1)
            evs[i + 1].record(s)
        torch.cuda.synchronize()
        return [round(evs[i].elapsed_time(evs[i + 1]) * 1e3, 1) for i in range(n)]

    def clock():
        h.set_option("profile", 1)
        launch(1)
        torch.cuda.synchronize()
        cyc = h.stat("state_read_miss2") + h.stat("no_ready_but_valid")  # s_memtime cycles, loader wave 0
        act = h.stat("state_active")  # s_memrealtime ticks x nominal clock -> nominal cycles
        h.set_option("profile", 0)
        return {"loader_cycles": cyc, "nominal_cycles": act, "clock_ratio": round(cyc / max(act, 1), 4)}

    def busy_copy(sec):
        a = torch.empty(1 << 27, dtype=torch.float64, device="cuda")
        b = torch.empty_like(a)
        t = time.perf_counter()
        while time.perf_counter() - t < sec:
            for _ in range(8):
                b.copy_(a)
            torch.cuda.synchronize()
        del a, b

    def busy_spmv(sec):
        t = time.perf_counter()
        while time.perf_counter() - t < sec:
            launch(50)
            torch.cuda.synchronize()

    launch(5)
    torch.cuda.synchronize()
    out["A_bench_like_20"] = pair(20)
    out["B_each_20"] = each(20)
    time.sleep(1.0)
    out["C_after_idle_20"] = pair(20)
    out["D_300"] = pair(300)
    out["D_then_20"] = pair(20)
    out["D_each_20"] = each(20)
    time.sleep(1.0)
    busy_copy(0.5)
    out["E_after_copy_20"] = pair(20)
    time.sleep(1.0)
    busy_spmv(0.5)
    out["F_after_spmv_20"] = pair(20)
    out["F_each_20"] = each(20)
    time.sleep(1.0)
    out["G_clock_after_idle"] = clock()
    launch(300)
    out["G_clock_after_300"] = clock()
    print(json.dumps(out), flush=True)
    h.close()


if __name__ == "__main__":
    main()
