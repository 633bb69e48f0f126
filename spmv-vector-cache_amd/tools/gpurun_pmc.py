import sys; sys.path.insert(0, 'spmv-vector-cache_amd')
import numpy as np, torch, hipspmv as hs
# gpurun_pmc.py KERNEL [c3|c4|c4sK|c5sK]: 10 launches of KERNEL on the workload (the
# child program of tools/gpurun_pmc.sh's rocprofv3 --pmc passes)
kernel = sys.argv[1] if len(sys.argv) > 1 else "vcache_split"
w = sys.argv[2] if len(sys.argv) > 2 else "c3"
if w.startswith("c5s"):  # C5 shard k of 8 (R-MAT scale 24, the library's partition), as bench.py cuts it
    k, n = int(w[3:]), 1 << 24
    rp, ci, v = hs.gen_rmat_csr(24)
    b = hs.partition_rows_cost(rp, ci, n, 8)
    r0, r1 = int(b[k]), int(b[k + 1])
    e0, e1 = int(rp[r0]), int(rp[r1])
    h = hs.Handle.from_csr((rp[r0:r1 + 1].astype(np.int64) - e0).astype(np.uint32), ci[e0:e1].copy(),
                           v[e0:e1].copy(), r1 - r0, n)
    rows = r1 - r0
    print("alg_bytes", h.stat("alg_bytes"), "rows", rows, "nnz", e1 - e0, flush=True)
elif w.startswith("c4s"):  # C4 shard k of 8: rows [k 2^21, (k+1) 2^21) of the 2^24 x 2^24 stripe matrix
    k, n = int(w[3:]), 1 << 24
    rows = n // 8
    rp, ci, v = hs.gen_stripe_csr(k * rows, rows, n, 32)
    h = hs.Handle.from_csr(rp, ci, v, rows, n)
    print("alg_bytes", h.stat("alg_bytes"), "rows", rows, "nnz", ci.size, flush=True)
else:
    n = 1 << (24 if w == "c4" else 20)
    rp, ci, v = hs.gen_stripe_csr(0, n, n, 32)
    h = hs.Handle.from_csr(rp, ci, v, n, n)
    rows = n
del rp, ci, v
x = torch.from_numpy(hs.gen_vector(n, 3)).cuda(); y = torch.empty(rows, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
h.set_kernel(kernel)
mode = hs.MODE_FAST if any(k in kernel for k in ("split", "vector", "wcsr", "flow")) else hs.MODE_ORDERED
for _ in range(10): h.exec_device(x, y, beta=0, mode=mode, stream=s)
torch.cuda.synchronize()
print("ran", h.kernel_name(mode), "x10", flush=True)
