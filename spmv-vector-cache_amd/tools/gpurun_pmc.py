import sys; sys.path.insert(0, 'spmv-vector-cache_amd')
import numpy as np, torch, hipspmv as hs
# gpurun_pmc.py KERNEL [c3|c4]: 10 launches of KERNEL on the workload (the
# child program of tools/gpurun_pmc.sh's rocprofv3 --pmc passes)
kernel = sys.argv[1] if len(sys.argv) > 1 else "vcache_split"
n = 1 << (24 if len(sys.argv) > 2 and sys.argv[2] == "c4" else 20)
rp, ci, v = hs.gen_stripe_csr(0, n, n, 32)
h = hs.Handle.from_csr(rp, ci, v, n, n)
del rp, ci, v
x = torch.from_numpy(hs.gen_vector(n, 3)).cuda(); y = torch.empty(n, dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
h.set_kernel(kernel)
mode = hs.MODE_FAST if "split" in h.kernel_name(hs.MODE_FAST) or "vector" in h.kernel_name(hs.MODE_FAST) else hs.MODE_ORDERED
for _ in range(10): h.exec_device(x, y, beta=0, mode=mode, stream=s)
torch.cuda.synchronize()
print("ran", h.kernel_name(mode), "x10", flush=True)
