// Probe: per-CU throughput of streaming a shared 8 MB x vector into LDS in
// panels (what the vcache kernel does per row block), by staging method.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: register staged (global_load_dwordx4 -> ds_write_b128), prefetch 1 panel
// MODE 1: loads only (no LDS), xor-accumulated to stay live
// MODE 2: LDS-DMA global_load_lds_dwordx4
template <int MODE, int PB /*panel bytes*/, int NT>
__global__ __launch_bounds__(NT) void k_xs(const u32x4* __restrict__ x, uint32_t npanels, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[2][PB / 4];
  constexpr int V = PB / 16 / NT;  // 16-byte vectors per thread per panel
  const int t = threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[V], n[V];
  if (MODE != 2) {
#pragma unroll
    for (int j = 0; j < V; ++j) r[j] = x[t + j * NT];
  }
  for (uint32_t p = 0; p < npanels; ++p) {
    const u32x4* src = x + (size_t)((p + 1) % npanels) * (PB / 16);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < V; ++j) n[j] = src[t + j * NT];
#pragma unroll
      for (int j = 0; j < V; ++j) *reinterpret_cast<u32x4*>(&lds[p & 1][4 * (t + j * NT)]) = r[j];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = n[j];
    } else if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < V; ++j) { u32x4 v = src[t + j * NT]; acc ^= v; }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(src + t + j * NT),
                                         (__attribute__((address_space(3))) void*)&lds[p & 1][4 * (j * NT + (t & ~63))], 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if (MODE == 1) { if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1; }
  else if (t == 0) out[blockIdx.x] = lds[0][5] + lds[1][7];
}

template <typename F> double time_us(F f, int reps = 20) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  std::vector<float> t;
  for (int i = 0; i < reps; ++i) { CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1000.f); }
  std::sort(t.begin(), t.end()); return t[t.size() / 2];
}

int main() {
  const size_t XB = 8u << 20;
  u32x4* x; uint32_t* out;
  CK(hipMalloc(&x, XB)); CK(hipMemset(x, 1, XB)); CK(hipMalloc(&out, 4096 * 4));
  auto rep = [&](const char* nm, int grid, uint32_t np, uint32_t pb, double us) {
    double per_cu = (double)np * pb * grid / 256.0;
    printf("%-44s grid=%4d %8.2f us  per-CU %6.1f GB/s  chip %7.1f GB/s\n", nm, grid, us, per_cu / us * 1e-3,
           (double)np * pb * grid / us * 1e-3);
  };
  const uint32_t np64 = XB / 65536;
  rep("regstage 64KB panels 1024thr", 256, np64, 65536, time_us([&] { k_xs<0, 65536, 1024><<<256, 1024>>>(x, np64, out); }));
  rep("loads-only 64KB 1024thr", 256, np64, 65536, time_us([&] { k_xs<1, 65536, 1024><<<256, 1024>>>(x, np64, out); }));
  rep("lds-dma 64KB 1024thr", 256, np64, 65536, time_us([&] { k_xs<2, 65536, 1024><<<256, 1024>>>(x, np64, out); }));
  const uint32_t np32 = XB / 32768;
  rep("regstage 32KB panels 1024thr", 256, np32, 32768, time_us([&] { k_xs<0, 32768, 1024><<<256, 1024>>>(x, np32, out); }));
  rep("lds-dma 32KB 1024thr", 256, np32, 32768, time_us([&] { k_xs<2, 32768, 1024><<<256, 1024>>>(x, np32, out); }));
  rep("regstage 32KB 512thr x2/CU", 512, np32, 32768, time_us([&] { k_xs<0, 32768, 512><<<512, 512>>>(x, np32, out); }));
  rep("lds-dma 32KB 512thr x2/CU", 512, np32, 32768, time_us([&] { k_xs<2, 32768, 512><<<512, 512>>>(x, np32, out); }));
  rep("loads-only 32KB 512thr x2/CU", 512, np32, 32768, time_us([&] { k_xs<1, 32768, 512><<<512, 512>>>(x, np32, out); }));
  const uint32_t np16 = XB / 16384;
  rep("lds-dma 16KB 256thr x4/CU", 1024, np16, 16384, time_us([&] { k_xs<2, 16384, 256><<<1024, 256>>>(x, np16, out); }));
  rep("loads-only 16KB 256thr x8/CU", 2048, np16, 16384, time_us([&] { k_xs<1, 16384, 256><<<2048, 256>>>(x, np16, out); }));
  return 0;
}
