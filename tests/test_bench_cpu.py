"""bench.py's host logic on CPU: the HIP handle and the torch.cuda surface are
replaced by stand-ins (the handle computes y with the oracle), so the contract
JSON, the timing/parity/roofline/cpu_baseline legs and the N>1 code path
(gloo, world size 2) are exercised without a GPU.  The real kernels are
covered by the -m gpu tests; this only guards the script itself."""
import contextlib
import io
import json
import os
import sys
import time
from contextlib import redirect_stdout

import numpy as np
import pytest
import torch

import hipspmv as hs
import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeHandle:
    def __init__(self, rowptr, colind, vals, rows, cols, device=0):
        self.rows, self.cols = rows, cols
        self.colptr, self.rowind, self.cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        self.nnz = colind.size
        self.kernel = "auto"

    @classmethod
    def from_csr(cls, rowptr, colind, vals, rows, cols, device=0):
        return cls(rowptr, colind, vals, rows, cols, device)

    def set_kernel(self, k):
        self.kernel = k

    def set_option(self, key, value):
        self.opts = getattr(self, "opts", {})
        self.opts[key] = value

    def kernel_name(self, mode):
        return "vcache_split" if mode == hs.MODE_FAST else "vcache"

    def exec_device(self, x, y_out, y_in=None, beta=0, mode=hs.MODE_ORDERED, stream=None):
        y = oracle.spmv_csc(self.colptr, self.rowind, self.cvals, x.numpy(), rows=self.rows)
        y_out.copy_(torch.from_numpy(y))

    def stat(self, key):
        if key == "setup_ns":
            return 1000
        if key.startswith("setup_") and key.endswith("_ns"):  # create's phases
            return 250
        if key == "wcsr_segments":
            return 0
        if key == "resident_entry_bytes":  # the library's default: about half a vcache layout's entries
            return 6 * self.nnz
        assert key == "alg_bytes"
        return 12 * self.nnz + 4 * (self.rows + 1) + 8 * self.cols + 8 * self.rows

    def close(self):
        pass


class FakeEvent:
    def __init__(self, enable_timing=True):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class FakeStream:
    cuda_stream = 0


def _patch(monkeypatch):
    import bench
    monkeypatch.setattr(bench.hs.Handle, "from_csr", FakeHandle.from_csr)
    monkeypatch.setattr(bench.hs, "release_wait", lambda: None)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: FakeStream())
    monkeypatch.setattr(torch.cuda, "Event", FakeEvent)
    real_device = torch.device
    monkeypatch.setattr(bench.torch, "device", lambda *a, **k: real_device("cpu"))
    monkeypatch.setattr(bench, "COPY_BYTES", 1 << 20)
    # the profiler leg starts a child bench on the GPU: its plumbing has its own test below
    monkeypatch.setattr(bench, "rocprof_leg", lambda a: {"kernel": "hipspmv::k_fake", "calls": 3, "avg_us": 1.0})
    monkeypatch.setattr(bench, "pmc_leg", lambda a: "no GPU: the PMC leg has its own test below")
    # no HIP graph capture on the CPU stand-in: the timed region runs plain launches
    monkeypatch.setattr(torch.cuda, "Stream", lambda *a, **k: FakeStream())
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())

    class NoGraph:
        def __init__(self):
            raise RuntimeError("no HIP graphs on the CPU stand-in")
    monkeypatch.setattr(torch.cuda, "CUDAGraph", NoGraph)
    return bench


def _run(bench, argv):
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    buf = io.StringIO()
    try:
        with redirect_stdout(buf):
            bench.main()
    finally:
        sys.argv = old
    lines = [l for l in buf.getvalue().splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def test_bench_json_contract_single(monkeypatch):
    sys.path.insert(0, REPO)
    bench = _patch(monkeypatch)
    out = _run(bench, ["--steps", "2", "--warmup", "1", "--log2-rows", "12", "--log2-cols", "12",
                       "--cpu-seconds", "0.05", "--strong-scale", "12", "--c5-scale", "14", "--c5-steps", "2"])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in out, key
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["scaling"] == "weak" and out["dtype"] == "f64"
    assert out["config"]["workload"].startswith("C3") and out["config"]["mode"] == "fast"
    rf = out["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0 and abs(rf["frac"] - rf["achieved"] / 8000.0) < 1e-3
    cb = out["cpu_baseline"]
    assert cb["cores"] == 1 and cb["kind"] == "port" and cb["value"] > 0
    assert rf["measured_copy_gbs"] >= 0 and rf["kernel_us_per_launch"]["launches"] == 2
    assert rf["kernel_us_per_launch"]["min"] <= rf["kernel_us_per_launch"]["median"] <= rf["kernel_us_per_launch"]["max"]
    assert out["pcie_us"]["x_h2d"] >= 0 and out["pcie_us"]["y_d2h"] >= 0
    mt = out["cpu_baseline_all_cores"]
    assert mt["cores"] >= 1 and mt["value"] > 0 and mt["bit_exact_vs_softwarespmv"]
    # the stand-in computes the ordered result, so both legs must pass their parity checks
    assert out["parity"].startswith("within FAST bound")
    assert out["secondary"]["mode"] == "ordered" and out["secondary"]["parity"] == "bit-exact vs oracle"
    prov = rf["kernel_provenance"]  # the stand-in reports vcache_split: the real library's fingerprint
    assert prov["same_as_gpu_validated_build"] is True and prov["kernel"].startswith("void hipspmv::k_vcache<double, 3")
    rp = out["rocprof"]
    assert rp["kernel"] == "hipspmv::k_fake" and rp["event_kernel_us"] == rf["kernel_us"]
    assert abs(rp["event_over_rocprof"] - rf["kernel_us"] / 1.0) < 1e-3
    # per-rank parity (sampled rows of the shard, both modes) and the C4 strong block beside the headline
    (rp0,) = out["rank_parity"]
    assert rp0["rank"] == 0 and rp0["fast"].startswith("within FAST bound") and rp0["ordered"].startswith("bit-exact")
    st = out["strong"]
    assert st["scaling"] == "strong" and st["nnz_total"] == 32 << 12 and st["rows_per_rank"] == 1 << 12
    assert st["rank_parity"][0].startswith("within FAST bound") and len(st["rank_kernel_us"]) == 1
    assert out["gen_s"] >= 0 and out["setup_s"] >= 0 and out["setup_ns_lib"] == 1000
    # the C5 block: 8 cost-balanced shards of R-MAT scale 12, each timed and checked against the oracle
    c5 = out["c5_shards"]
    assert len(c5["shards"]) == 8 and c5["nnz_total"] == sum(s["nnz"] for s in c5["shards"])
    assert c5["shards"][0]["rows"][0] == 0 and c5["shards"][-1]["rows"][1] == 1 << 14
    assert all(s["parity"].startswith("within FAST bound") for s in c5["shards"] if s["kernel"]), c5
    assert c5["max_over_min"] >= 1.0 and c5["value"] > 0
    # the residency share of the headline and the C4 shard block
    assert rf["resident_entry_bytes"] == 6 * (32 << 12) and 0 < rf["frac_no_residency"]
    assert rf["kernel_us_no_residency"] > 0 and "vcache_nt 0" in rf["no_residency_control"]
    c4 = out["c4_shards"]
    assert [s["shard"] for s in c4["shards"]] == [0, 7] and c4["min_roofline_frac"] > 0
    assert c4["shards"][0]["rows"][0] == 0 and c4["shards"][1]["rows"][1] == 1 << 12
    assert all(s["parity"].startswith("within FAST bound") for s in c4["shards"]), c4


FAKE_ROCPROF = """#!/usr/bin/env python3
import os, sys
args = sys.argv[1:]
assert args[:2] == ["--kernel-trace", "--stats"], args
sep = args.index("--")
prog = args[sep + 1:]
# the program itself follows "--" (no env/sh/launcher hop), in child mode
assert os.path.basename(prog[0]).startswith("python") and prog[1].endswith("bench.py"), prog
assert "--rocprof-child" in prog and "--no-cpu-baseline" in prog, prog
d = args[args.index("-d") + 1]
os.makedirs(os.path.join(d, "host", "123"), exist_ok=True)
with open(os.path.join(d, "host", "123", "run_kernel_stats.csv"), "w") as f:
    f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\\n')
    f.write('"void hipspmv::k_vcache<double, 2>(int)",106,15264000,144000.0,99.0,139000,149000,1700.0\\n')
    f.write('"__amd_rocclr_copyBuffer",15,50282,3352.1,0.5,2601,4440,657.3\\n')
"""


def test_rocprof_leg_plumbing(tmp_path, monkeypatch):
    """The profiler leg: rocprofv3 with --kernel-trace --stats only, the bench
    itself right after "--" in child mode, and the dominant hipspmv kernel read
    back from kernel_stats.csv (a fake rocprofv3 here; no GPU is touched)."""
    import argparse
    import shutil
    sys.path.insert(0, REPO)
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF)
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda name: str(fake) if name == "rocprofv3" else None)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    a = argparse.Namespace(steps=200, workload="c3", scale=24, log2_rows=20, log2_cols=20, nnz_per_row=32,
                           kernel="auto", mode="fast", vcache_xlane=-1, vcache_dma=-1, vcache_map=0,
                           rocprof_timeout=60.0)
    s = bench.rocprof_leg(a)
    assert "error" not in s, s
    assert s["kernel"].startswith("void hipspmv::k_vcache") and s["calls"] == 106
    assert s["avg_us"] == 144.0 and s["min_us"] == 139.0 and s["max_us"] == 149.0
    assert s["csv"].endswith("run_kernel_stats.csv") and s["tool"] == "rocprofv3 --kernel-trace --stats"


FAKE_ROCPROF_PMC = """#!/usr/bin/env python3
import os, sys
args = sys.argv[1:]
assert args[0] == "--pmc" and len(args[1].split()) == 1, args  # one counter per pass, its own run
assert "--kernel-trace" not in args and "--stats" not in args and "-s" not in args, args
sep = args.index("--")
prog = args[sep + 1:]
assert os.path.basename(prog[0]).startswith("python") and prog[1].endswith("bench.py"), prog
assert "--rocprof-child" in prog and "--no-secondary" in prog, prog
d = args[args.index("-d") + 1]
os.makedirs(os.path.join(d, "host", "9"), exist_ok=True)
val = {"FETCH_SIZE": 200000.0, "WRITE_SIZE": 16384.0}[args[1]]
with open(os.path.join(d, "host", "9", "run_counter_collection.csv"), "w") as f:
    f.write("Correlation_Id,Dispatch_Id,Agent_Id,Queue_Id,Process_Id,Thread_Id,Grid_Size,Kernel_Id,Kernel_Name,"
            "Workgroup_Size,LDS_Block_Size,Scratch_Size,VGPR_Count,Accum_VGPR_Count,SGPR_Count,Counter_Name,"
            "Counter_Value\\n")
    for disp in (1, 2):
        f.write(f'{disp},{disp},1,1,1,1,262144,7,"void hipspmv::k_vcache<double, 2>(int)",1024,163840,0,88,0,'
                f'40,{args[1]},{val}\\n')
"""


def test_pmc_leg_traffic(tmp_path, monkeypatch):
    """The traffic leg: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over the bench in child mode;
    traffic = FETCH_SIZE KB x 1024 x 2 + WRITE_SIZE KB x 1024 per launch (a fake rocprofv3; no GPU)."""
    import argparse
    import shutil
    sys.path.insert(0, REPO)
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text(FAKE_ROCPROF_PMC)
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda name: str(fake) if name == "rocprofv3" else None)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    a = argparse.Namespace(steps=200, workload="c3", scale=24, log2_rows=20, log2_cols=20, nnz_per_row=32,
                           kernel="auto", mode="fast", vcache_xlane=-1, vcache_dma=-1, vcache_map=0,
                           rocprof_timeout=60.0)
    files = bench.pmc_leg(a)
    assert isinstance(files, list) and len(files) == 2, files
    assert bench.traffic_from_csv(files, "k_vcache") == 200000.0 * 1024 * 2 + 16384.0 * 1024


def test_rocprof_leg_timeout_kills_child(tmp_path, monkeypatch):
    import argparse
    import shutil
    sys.path.insert(0, REPO)
    import bench
    fake = tmp_path / "rocprofv3"
    fake.write_text("#!/bin/sh\nsleep 60\n")
    fake.chmod(0o755)
    monkeypatch.setattr(shutil, "which", lambda name: str(fake) if name == "rocprofv3" else None)
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    a = argparse.Namespace(steps=5, workload="c3", scale=24, log2_rows=20, log2_cols=20, nnz_per_row=32,
                           kernel="auto", mode="fast", vcache_xlane=-1, vcache_dma=-1, vcache_map=0,
                           rocprof_timeout=1.0)
    t = time.perf_counter()
    s = bench.rocprof_leg(a)
    assert "timed out" in s["error"] and time.perf_counter() - t < 10


def test_kernel_stats_summary_committed_profile():
    """The parser on the committed round-1 table (kernel_stats.csv layout)."""
    sys.path.insert(0, REPO)
    import bench
    s = bench.kernel_stats_summary(os.path.join(REPO, "profiles", "r01", "kernel_stats_from_pmc.csv"))
    assert "k_vcache<double, 2" in s["kernel"] and s["calls"] == 65 and abs(s["avg_us"] - 144.814) < 1e-3


def _rank_main(rank, world, store_path, q, extra=()):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT="0")
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "spmv-vector-cache_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import torch.distributed as dist

    class MP:  # minimal monkeypatch
        def setattr(self, obj, name, val):
            setattr(obj, name, val)

    bench = _patch(MP())
    real_init = dist.init_process_group
    # file rendezvous: no TCP port to race for between consecutive tests
    dist.init_process_group = lambda backend, device_id=None: real_init(
        "gloo", init_method=f"file://{store_path}", rank=rank, world_size=world)
    try:
        out = _run(bench, ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--log2-rows", "10",
                           "--log2-cols", "10", "--strong-scale", "11", "--parity-rows", "300", *extra])
    except BaseException as e:  # report it to the parent instead of a bare exit code
        q.put((rank, f"ERROR: {type(e).__name__}: {e}"))
        raise
    q.put((rank, out))


def _multi_rank(extra, world=2):
    import multiprocessing as mp
    import tempfile
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = os.path.join(tempfile.mkdtemp(prefix="bench_gloo_"), "store")
    procs = [ctx.Process(target=_rank_main, args=(r, world, store, q, tuple(extra))) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    errors = [v for v in res.values() if isinstance(v, str)]
    assert not errors, errors
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


@pytest.mark.parametrize("workload,scale", [("c4", 11), ("c5", 10)])
def test_bench_strong_workloads_single(monkeypatch, workload, scale):
    sys.path.insert(0, REPO)
    bench = _patch(monkeypatch)
    out = _run(bench, ["--steps", "2", "--warmup", "1", "--workload", workload, "--scale", str(scale),
                       "--cpu-seconds", "0.05", "--cpu-sample-nnz", "5000"])
    assert out["scaling"] == "strong" and out["config"]["workload"].startswith(workload.upper())
    assert out["config"]["rows_per_gpu"] == 1 << scale
    assert out["config"]["nnz_total"] == out["config"]["nnz_per_gpu"]
    assert out["parity"].startswith("within FAST bound") and "first" in out["cpu_baseline"]["sample"]


@pytest.mark.parametrize("workload,scale", [("c4", 11), ("c5", 10)])
def test_bench_strong_workloads_gloo(workload, scale):
    res = _multi_rank(["--workload", workload, "--scale", str(scale)])
    out = res[0]
    assert res[1] is None and out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert len(out["rank_kernel_us"]) == 2
    assert out["y_allgather_us"] > 0 and out["iterative"]["value"] <= out["value"]
    # the two shards together are the whole matrix
    if workload == "c4":
        assert out["config"]["nnz_total"] == 32 << scale and out["config"]["rows_per_gpu"] == 1 << (scale - 1)
    else:
        import hipspmv as hs_
        assert out["config"]["nnz_total"] == hs_.gen_rmat_csr(scale)[1].size


def _check_rank_parity_and_strong(out, world):
    rp = out["rank_parity"]
    assert [p["rank"] for p in rp] == list(range(world))
    assert all(p["fast"].startswith("within FAST bound") and p["ordered"].startswith("bit-exact") for p in rp), rp
    # the shards tile the rows: rank r owns [r*2^10, (r+1)*2^10)
    assert [p["rows"] for p in rp] == [[r << 10, (r + 1) << 10] for r in range(world)]
    st = out["strong"]  # the C4 (here 2^11) matrix cut into `world` row blocks
    assert st["scaling"] == "strong" and st["nnz_total"] == 32 << 11 and st["rows_per_rank"] == (1 << 11) // world
    assert len(st["rank_kernel_us"]) == world and len(st["rank_parity"]) == world
    assert all(p.startswith("within FAST bound") for p in st["rank_parity"]), st["rank_parity"]
    assert st["x_bcast_us"] > 0 and st["value"] > 0


def test_bench_multi_rank_gloo():
    res = _multi_rank([])
    assert res[1] is None  # only rank 0 prints the line
    out = res[0]
    _check_rank_parity_and_strong(out, 2)
    assert out["n_gpus"] == 2 and out["x_bcast_us"] is not None
    e2e = out["end_to_end"]
    assert e2e["value"] <= out["value"] and abs(e2e["ms_per_step"] - out["ms_per_step"] - out["x_bcast_us"] * 1e-3) < 1e-3
    assert out["config"]["parallelism"].startswith("row-partition x2")
    # value is the whole-job rate: both ranks' flops over the max step time
    # value is rounded to 0.01 GFLOP/s: tiny CPU rates need the half-unit on top of 2 %
    assert abs(out["value"] - 2 * 2 * out["config"]["nnz_per_gpu"] / (out["ms_per_step"] * 1e-3) / 1e9) < \
        0.02 * out["value"] + 0.006


def test_bench_four_ranks_gloo():
    # more ranks than the GPU tests can use: rank r owns rows [r*2^10, (r+1)*2^10)
    res = _multi_rank([], world=4)
    out = res[0]
    assert all(res[r] is None for r in (1, 2, 3))
    assert out["n_gpus"] == 4 and len(out["rank_kernel_us"]) == 4
    _check_rank_parity_and_strong(out, 4)
    assert out["config"]["nnz_total"] == 4 * out["config"]["nnz_per_gpu"]


@pytest.mark.parametrize("workload,scale", [("c4", 12), ("c5", 12)])
def test_bench_eight_ranks_gloo(workload, scale):
    # the driver's N=8 case rehearsed on CPU: the C4 / C5
    # strong-scaled workloads cut into eight row blocks, the x broadcast and the
    # y allgather timed, per-rank parity on every rank
    res = _multi_rank(["--workload", workload, "--scale", str(scale)], world=8)
    out = res[0]
    assert all(res[r] is None for r in range(1, 8))
    assert out["n_gpus"] == 8 and out["scaling"] == "strong" and len(out["rank_kernel_us"]) == 8
    assert out["x_bcast_us"] is not None and out["x_bcast_us"] > 0
    assert out["y_allgather_us"] is not None and out["y_allgather_us"] > 0
    assert out["end_to_end"] is not None and out["end_to_end"]["value"] <= out["value"]
    assert out["iterative"] is not None and out["iterative"]["value"] <= out["value"]
    rp = out["rank_parity"]
    assert [p["rank"] for p in rp] == list(range(8))
    assert all(p["fast"].startswith("within FAST bound") and p["ordered"].startswith("bit-exact") for p in rp), rp
    rows = [p["rows"] for p in rp]  # the blocks tile the matrix
    assert rows[0][0] == 0 and rows[-1][1] == 1 << scale and all(rows[i][1] == rows[i + 1][0] for i in range(7))
    assert "strong" in out["scaling_note"]
    if workload == "c5":
        import hipspmv as hs_
        rp_, ci_, _ = hs_.gen_rmat_csr(scale)
        assert out["config"]["nnz_total"] == ci_.size
        # the blocks are the library's partition (hipspmv_partition_rows), not the bench's
        assert [r[0] for r in rows] == [int(b) for b in hs_.partition_rows_cost(rp_, ci_, 1 << scale, 8)[:8]]
