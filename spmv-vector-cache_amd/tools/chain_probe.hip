// chain_probe: how fast can one wave add a row's products in sequence?
//
// ORDERED mode sums every row in ascending column order, each add rounded
// (SoftwareSpMV.cpp:62), so a hub row of n entries is a chain of n dependent
// f64 adds however many waves compute its products.  This probe times the
// chain alone (one wave, s_memtime cycles per add) in the forms a kernel can
// feed it:
//   reg     : products already in the adding lane's registers (the floor)
//   readlane: products spread over the wave's 64 lanes, fetched in order with
//             v_readlane (k_sell's hub-row ORDERED form today)
//   lds     : products in LDS, read by the adding lane with ds_read_b128
//             (two per read, reads issued ahead of the adds)
// Prints cycles per add and the implied time for a 238,554-entry row (the
// longest row of R-MAT scale 24, config C5) at 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

constexpr int kN = 1 << 16;  // adds per chain

__global__ __launch_bounds__(64) void k_reg(const double* __restrict__ in, double* out, unsigned long long* cyc) {
#pragma clang fp contract(off)
  double r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = in[threadIdx.x * 16 + i];
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kN / 16; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = acc + r[i];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ __launch_bounds__(64) void k_readlane(const double* __restrict__ in, double* out,
                                                 unsigned long long* cyc) {
#pragma clang fp contract(off)
  const double p = in[threadIdx.x];
  const unsigned long long pb = __builtin_bit_cast(unsigned long long, p);
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kN / 64; ++it) {
#pragma unroll
    for (int l = 0; l < 64; ++l) {
      const unsigned long long v = (unsigned long long)(unsigned)__builtin_amdgcn_readlane((unsigned)pb, l) |
                                   ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((unsigned)(pb >> 32), l)
                                    << 32);
      acc = acc + __builtin_bit_cast(double, v);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ __launch_bounds__(64) void k_lds(const double* __restrict__ in, double* out, unsigned long long* cyc) {
#pragma clang fp contract(off)
  __shared__ double buf[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) buf[i] = in[i];
  __syncthreads();
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    for (int it = 0; it < kN / 4096; ++it) {
      for (int i = 0; i < 4096; i += 16) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
          const double2 w = *reinterpret_cast<const double2*>(&buf[i + k]);
          v[k] = w.x;
          v[k + 1] = w.y;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) acc = acc + v[k];
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// dpp: k_sell's ORDERED hub chain (csrc/sell.hip hub_row_exact): 8 products
// per lane, 64 steps of 8 dependent adds then a DPP wave rotation handing the
// sum to the next lane
__device__ __forceinline__ double ror1(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, 0x13C, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x13C, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__global__ __launch_bounds__(64) void k_dpp(const double* __restrict__ in, double* out, unsigned long long* cyc) {
#pragma clang fp contract(off)
  double p[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = in[threadIdx.x * 8 + j];
  double acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kN / 512; ++it) {
#pragma unroll
    for (int l = 0; l < 64; ++l) {
      double s = acc;
#pragma unroll
      for (int j = 0; j < 8; ++j) s = s + p[j];
      acc = ror1(s);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <typename K>
static void run(const char* nm, K kern, const double* din, double* dout, unsigned long long* dcyc) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, din, dout, dcyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
    best = c < best ? c : best;
  }
  const double per = (double)best / kN;
  std::printf("%-9s %6.2f cycles per dependent add -> 238554-entry row: %7.1f us at 2.4 GHz\n", nm, per,
              per * 238554 / 2400.0);
}

int main() {
  double* din;
  double* dout;
  unsigned long long* dcyc;
  CK(hipMalloc(&din, 8 * 4096));
  CK(hipMalloc(&dout, 8 * 64));
  CK(hipMalloc(&dcyc, 8));
  double h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 1.0 + i * 1e-6;
  CK(hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice));
  run("reg", k_reg, din, dout, dcyc);
  run("readlane", k_readlane, din, dout, dcyc);
  run("lds", k_lds, din, dout, dcyc);
  run("dpp8", k_dpp, din, dout, dcyc);
  return 0;
}
