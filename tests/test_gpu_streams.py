"""GPU: stream lifetime and handle release.

* Every stream a handle launches on gets its own combine scratch set, so no
  launch records or waits on another stream's event: a stream may be destroyed
  right after its last launch (include/hipspmv.h, hipspmv_exec_device).
* hipspmv_destroy returns at once; the release thread frees the handle's
  memory once the device has finished the work queued before the destroy.

Results are checked bit for bit against a launch on torch's current stream
(vcache_split is deterministic) and that launch against the oracle's FAST
bound.
"""
import ctypes as C
import time

import numpy as np
import pytest

import hipspmv as hs
import oracle

pytestmark = pytest.mark.gpu


def _hip():
    lib = C.CDLL("libamdhip64.so")
    lib.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    lib.hipStreamDestroy.argtypes = [C.c_void_p]
    lib.hipStreamSynchronize.argtypes = [C.c_void_p]
    lib.hipStreamQuery.argtypes = [C.c_void_p]
    for f in ("hipStreamCreate", "hipStreamDestroy", "hipStreamSynchronize", "hipStreamQuery"):
        getattr(lib, f).restype = C.c_int
    return lib


def _raw_stream(lib):
    s = C.c_void_p()
    assert lib.hipStreamCreate(C.byref(s)) == 0
    return s.value


def _c3_like(n=1 << 16, seed=0):
    rowptr, colind, vals = hs.gen_stripe_csr(seed, n, n, 32)
    return n, rowptr, colind, vals


def _reference_bits(h, n, x):
    import torch
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    return y.cpu().numpy()


def _within_fast_bound(n, rowptr, colind, vals, x, y):
    colptr, rowind, cvals = oracle.csr2csc(n, n, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, x, rows=n)
    absprod = np.zeros(n)
    lens = np.diff(rowptr.astype(np.int64))
    np.add.at(absprod, np.repeat(np.arange(n), lens), np.abs(vals * x[colind]))
    bound = 2.0 * np.maximum(lens, 1) * 2.0 ** -53 * absprod + 1e-300
    assert np.all(np.abs(y - y_ref) <= bound)


def test_launch_on_destroyed_side_stream_then_another(gpu):
    # a scratch kernel on a raw side stream A, A destroyed with the launch still queued, then
    # launches on streams B and C and on the handle's own stream (hipspmv_exec): each result is
    # the reference bits (nothing was recorded on A after its destruction; A's set is never reused
    # by B or C)
    import torch
    lib = _hip()
    n, rowptr, colind, vals = _c3_like()
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    h.set_kernel("vcache_split")
    xh = hs.gen_vector(n, 3)
    x = torch.from_numpy(xh).cuda()
    ref = _reference_bits(h, n, x)
    _within_fast_bound(n, rowptr, colind, vals, xh, ref)
    ys = [torch.full((n,), float("nan"), dtype=torch.float64, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    a = _raw_stream(lib)
    for _ in range(3):
        h.exec_device(x, ys[0], beta=0, mode=hs.MODE_FAST, stream=a)
    assert lib.hipStreamDestroy(a) == 0  # work still queued: the runtime finishes it
    b = _raw_stream(lib)
    h.exec_device(x, ys[1], beta=0, mode=hs.MODE_FAST, stream=b)
    c = _raw_stream(lib)
    h.exec_device(x, ys[2], beta=0, mode=hs.MODE_FAST, stream=c)
    h.exec_device(x, ys[3], beta=0, mode=hs.MODE_FAST, stream=b)
    y_host = h.exec(xh, beta=0, mode=hs.MODE_FAST)
    for s in (b, c):
        assert lib.hipStreamSynchronize(s) == 0
        assert lib.hipStreamDestroy(s) == 0
    torch.cuda.synchronize()
    assert y_host.tobytes() == ref.tobytes()
    for i, y in enumerate(ys):
        assert y.cpu().numpy().tobytes() == ref.tobytes(), i
    # current stream, A (destroyed), B, C, the handle's own: up to five stream values over four sets
    # (B may receive A's value once A's queue is gone: test_hip_stream_destroy_waits_for_queued_work)
    assert h.stat("scratch_streams") == 4 and h.stat("scratch_evictions") <= 1
    h.close()


def test_many_streams_evict_and_stay_exact(gpu):
    # six streams in turn, twice: sets are taken over least-recently-used after a device
    # synchronisation; every launch still gives the reference bits (u64 too: exact)
    import torch
    n, rowptr, colind, vals = _c3_like(seed=5)
    for dt in (np.float64, np.uint64):
        v = vals if dt == np.float64 else (vals.view(np.uint64) >> np.uint64(11))
        h = hs.Handle.from_csr(rowptr, colind, v, n, n)
        h.set_kernel("vcache_split")
        xh = hs.gen_vector(n, 7) if dt == np.float64 else np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        # u64 travels as int64 tensors (8-byte elements, the bits unchanged)
        x = torch.from_numpy(xh if dt == np.float64 else xh.view(np.int64)).cuda()
        y0 = torch.empty(n, dtype=torch.float64 if dt == np.float64 else torch.int64, device="cuda")
        h.exec_device(x, y0, beta=0, mode=hs.MODE_FAST, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        ref = y0.cpu().numpy().tobytes()
        if dt == np.uint64:
            colptr, rowind, cv = oracle.csr2csc(n, n, rowptr, colind, v)
            assert oracle.spmv_csc(colptr, rowind, cv, xh, rows=n).tobytes() == ref
        streams = [torch.cuda.Stream() for _ in range(6)]
        outs = [torch.empty_like(y0) for _ in range(12)]
        for k in range(12):
            h.exec_device(x, outs[k], beta=0, mode=hs.MODE_FAST, stream=streams[k % 6])
        torch.cuda.synchronize()
        for k in range(12):
            assert outs[k].cpu().numpy().tobytes() == ref, (dt, k)
        assert h.stat("scratch_evictions") >= 1
        h.close()


def test_wgather_split_concurrent_streams(gpu):
    # k_wgather_split's combine scratch (partials + share counters) is per stream like the vector
    # cache's: launches on three streams with nothing ordering them run at once and each gives the
    # reference bits, within the FAST bound of the oracle
    import torch
    rows, cols = 1 << 15, (1 << 21) + 7
    rowptr, colind, vals = hs.gen_stripe_csr(3, rows, cols, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, rows, cols)
    assert h.kernel_name(hs.MODE_FAST) == "wgather_split"
    xh = hs.gen_vector(cols, 9)
    x = torch.from_numpy(xh).cuda()
    y0 = torch.empty(rows, dtype=torch.float64, device="cuda")
    h.exec_device(x, y0, beta=0, mode=hs.MODE_FAST, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    ref = y0.cpu().numpy()
    colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
    y_ref = oracle.spmv_csc(colptr, rowind, cvals, xh, rows=rows)
    absprod = np.bincount(np.repeat(np.arange(rows), 32), weights=np.abs(vals * xh[colind]), minlength=rows)
    assert np.all(np.abs(ref - y_ref) <= 2.0 * 33 * 2.0 ** -53 * absprod + 1e-300)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.empty_like(y0) for _ in range(12)]
    for k in range(12):
        h.exec_device(x, outs[k], beta=0, mode=hs.MODE_FAST, stream=streams[k % 3])
    torch.cuda.synchronize()
    for k in range(12):
        assert outs[k].cpu().numpy().tobytes() == ref.tobytes(), k
    h.close()


def test_destroy_returns_without_waiting_for_the_device(gpu):
    # ~50 launches of a C3-sized vcache_split queued on a side stream; creating and destroying a
    # second handle meanwhile returns long before that queue drains (hipFree would have waited for
    # it: the round-5 1616 us outlier), the queued results are right, and release_wait completes
    import torch
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    assert h.kernel_name(hs.MODE_FAST) == "vcache_split"
    x = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    ref = _reference_bits(h, n, x)
    m, rp2, ci2, v2 = _c3_like(seed=9)
    h2 = hs.Handle.from_csr(rp2, ci2, v2, m, m)
    x2 = torch.from_numpy(hs.gen_vector(m, 4)).cuda()
    y2 = torch.empty(m, dtype=torch.float64, device="cuda")
    h2.exec_device(x2, y2, beta=0, mode=hs.MODE_FAST, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(side)
    for _ in range(50):
        h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=side)
    ev1.record(side)
    t0 = time.perf_counter()
    h2.exec_device(x2, y2, beta=0, mode=hs.MODE_FAST, stream=side)  # h2's last launch, queued last
    h2.close()  # hipspmv_destroy
    dt_ms = (time.perf_counter() - t0) * 1e3
    pending = not ev1.query()
    torch.cuda.synchronize()
    queued_ms = ev0.elapsed_time(ev1)
    assert y.cpu().numpy().tobytes() == ref.tobytes()
    hs.release_wait()
    # the destroy returned while the queue was still running (~5 ms of launches)
    assert pending and dt_ms < queued_ms / 2, (dt_ms, queued_ms)
    h.close()
    hs.release_wait()


def test_borrowed_shard_outlives_nothing(gpu):
    # a MultiHandle's shard keeps its MultiHandle alive, and closing the MultiHandle invalidates
    # the shard: a later call raises instead of touching freed native memory
    rows, cols = 4096, 4096
    rowptr, colind, vals = hs.gen_stripe_csr(0, rows, cols, 8)
    sh = hs.MultiHandle(rowptr, colind, vals, rows, cols, [0, 0], csr=True).shard(0)
    assert sh.stat("rows") > 0  # the parent is still alive through the shard
    m = sh._parent
    m.close()
    with pytest.raises(hs.HipSpMVError):
        sh.stat("rows")


def test_hip_stream_destroy_waits_for_queued_work(gpu):
    # the library tells streams apart by their handle value (include/hipspmv.h): that is safe as
    # long as a destroyed stream's value cannot come back while launches queued on it still run --
    # hipStreamDestroy returning only after the queued work has finished makes that so
    import torch
    lib = _hip()
    n = 1 << 20
    rowptr, colind, vals = hs.gen_stripe_csr(0, n, n, 32)
    h = hs.Handle.from_csr(rowptr, colind, vals, n, n)
    x = torch.from_numpy(hs.gen_vector(n, 3)).cuda()
    ref = _reference_bits(h, n, x)
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    a = _raw_stream(lib)
    for _ in range(30):
        h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=a)
    t0 = time.perf_counter()
    assert lib.hipStreamDestroy(a) == 0
    destroy_ms = (time.perf_counter() - t0) * 1e3
    b = _raw_stream(lib)
    reused = b == a
    h.exec_device(x, y, beta=0, mode=hs.MODE_FAST, stream=b)
    assert lib.hipStreamSynchronize(b) == 0 and lib.hipStreamDestroy(b) == 0
    torch.cuda.synchronize()
    assert y.cpu().numpy().tobytes() == ref.tobytes()
    print(f"hipStreamDestroy with 30 queued C3 launches: {destroy_ms:.2f} ms; value reused: {reused}")
    # ~30 x 95 us queued: a destroy that returned before them must not have handed its value on
    assert destroy_ms > 1.5 or not reused, (destroy_ms, reused)
    h.close()
