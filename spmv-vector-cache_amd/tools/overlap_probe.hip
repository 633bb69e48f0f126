// overlap_probe: does the C3 split kernel's x stream cost time because the
// memory system cannot serve it beside the entry stream, or because the
// per-panel workgroup barrier couples the two?
//
// Skeletons of one 1024-thread workgroup per CU, 131,072 entries per unit
// (C3 / 256 CUs: u32 code + f64 value, non-temporal, DE-deep register ring),
// x parts of 2^20 / S doubles (L2-served, as the product's column parts):
//   E   entries only, every compute wave free-running (no barrier);
//   X   x panels only, WL loader waves, LDS-DMA into a ring, free-running;
//   EX  both at once, no barrier between them;
//   A   the barrier-free vector cache: an NS-slot x ring in LDS handed over by
//       LDS counters (landed / consumed per slot) instead of s_barrier, each
//       compute wave owns R/WC rows of the y block (no two waves touch one y
//       row, so nothing else needs a barrier) and applies its entries of
//       every panel (LDS x read, LDS y read-modify-write);
//   G   no x staging: every wave gathers x from global memory (L1/L2) for its
//       entries of the current panel, y block in LDS, waves kept within D
//       panels of each other by an LDS counter (D = 0: free-running).
// Prints HIP-event time per launch over back-to-back launches.  Results are
// meaningless sums (timing only).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

constexpr int kT = 1024, kNW = 16;
constexpr uint32_t kNE = 131072;  // entries per unit
constexpr uint32_t kCols = 1u << 20;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// ring loads the compiler's waitcnt pass does not see: the kernels wait with
// exact explicit counts (vmcnt retires in issue order)
__device__ __forceinline__ uint32_t ald_u32_nt(const uint32_t* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ double ald_f64_nt(const double* p) {
  double r;
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(r) : "v"(p) : "memory");
  return r;
}
__device__ __forceinline__ double ald_f64(const double* p) {
  double r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- E / X / EX: free-running roles
template <bool E, bool X, int WL, int P>
__global__ __launch_bounds__(kT) void k_free(const uint32_t* __restrict__ code, const double* __restrict__ vals,
                                             const double* __restrict__ x, double* __restrict__ out,
                                             uint32_t part_cols, int S) {
  __shared__ double xb[2][P];
  __shared__ double pad[12000];  // one workgroup per CU, as the product
  constexpr int WC = kNW - WL, CT = WC * 64, EPT = 2, DE = 4;
  const int t = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const uint32_t u = blockIdx.x, h = (u / 8) % (uint32_t)S;
  const double* xp = x + (size_t)h * part_cols;
  double acc = 0.0;
  if (w < WL) {
    if constexpr (X && WL > 0) {
      constexpr uint32_t PAIRS = P / 2, ND = (PAIRS + WL * 64 - 1) / (WL * 64);
      const uint32_t npan = part_cols / P;
      for (uint32_t p = 0; p < npan; ++p) {
        double* slot = xb[p & 1];
#pragma unroll
        for (uint32_t j = 0; j < ND; ++j) {
          const uint32_t c0 = (j * WL + w) * 64;
          if (c0 + lane < PAIRS)
            __builtin_amdgcn_global_load_lds((const void*)(xp + (size_t)p * P + 2 * (c0 + lane)),
                                             (lds_void*)(slot + 2 * c0), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ND) : "memory");  // the previous panel landed
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else if (E) {
    const int ct = t - WL * 64;
    const uint32_t* cu = code + (size_t)u * kNE;
    const double* vu = vals + (size_t)u * kNE;
    constexpr uint32_t STEP = EPT * CT;
    const uint32_t nsteps = (kNE + STEP - 1) / STEP;
    uint32_t C[DE][EPT];
    double V[DE][EPT];
    auto load = [&](uint32_t s, uint32_t* c, double* v) {
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const uint32_t i = min(s * STEP + j * CT + ct, kNE - 1);
        c[j] = __builtin_nontemporal_load(cu + i);
        v[j] = __builtin_nontemporal_load(vu + i);
      }
    };
#pragma unroll
    for (int d = 0; d < DE; ++d) load(d, C[d], V[d]);
    const uint32_t padded = (nsteps + DE - 1) / DE * DE;
    for (uint32_t b = 0; b < padded; b += DE) {
#pragma unroll
      for (int i = 0; i < DE; ++i) {
#pragma unroll
        for (int j = 0; j < EPT; ++j) acc += (double)C[i][j] * V[i][j];
        load(b + i + DE, C[i], V[i]);
      }
    }
  }
  pad[t] = acc + xb[t & 1][t];
  __syncthreads();
  if (t == 0) out[u] = pad[5] + pad[999];
}

// ---- A: barrier-free vector cache skeleton
// entries of unit u: [panel][compute wave][EPW], EPW <= 64 (one per lane)
template <int R, int NS, int P, int WL, int L, int DE>
__global__ __launch_bounds__(kT) void k_async(const uint32_t* __restrict__ code, const double* __restrict__ vals,
                                              const double* __restrict__ x, double* __restrict__ out,
                                              uint32_t part_cols, int S, uint32_t epw) {
  constexpr int WC = kNW - WL;
  constexpr uint32_t RW = R / WC;  // rows owned by a compute wave
  __shared__ double ylds[R];
  __shared__ double xr[NS][P];
  __shared__ uint32_t landed[NS], consumed[NS];
  const int t = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const uint32_t u = blockIdx.x, h = (u / 8) % (uint32_t)S;
  const double* xp = x + (size_t)h * part_cols;
  const uint32_t npan = part_cols / P;
  for (uint32_t i = t; i < R; i += kT) ylds[i] = 0.0;
  if (t < NS) landed[t] = consumed[t] = 0;
  __syncthreads();
  if (w < WL) {
    constexpr uint32_t PAIRS = P / 2, ND = (PAIRS + WL * 64 - 1) / (WL * 64);
    auto dma = [&](uint32_t p) {
      double* slot = xr[p % NS];
#pragma unroll
      for (uint32_t j = 0; j < ND; ++j) {
        const uint32_t c0 = (j * WL + w) * 64;
        if (c0 + lane < PAIRS)
          __builtin_amdgcn_global_load_lds((const void*)(xp + (size_t)p * P + 2 * (c0 + lane)),
                                           (lds_void*)(slot + 2 * c0), 16, 0, 0);
      }
    };
    // L panels in flight: issue p, then publish p - L once it landed
    for (uint32_t p = 0; p < npan + L; ++p) {
      if (p < npan) {
        if (p >= NS) {
          const uint32_t need = WC * (p / NS);
          while (lds_ld(&consumed[p % NS]) < need) __builtin_amdgcn_s_sleep(1);
        }
        dma(p);
      } else {
        asm volatile("s_nop 0" ::: "memory");
      }
      if (p >= L) {
        if (p < npan)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * ND) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) lds_add(&landed[(p - L) % NS], 1);
      }
    }
  } else {
    const uint32_t cw = w - WL;
    const size_t ubase = (size_t)u * npan * WC * epw;
    const uint32_t* cu = code + ubase + cw * epw;
    const double* vu = vals + ubase + cw * epw;
    const uint32_t stride = WC * epw;
    const uint32_t last = (npan - 1) * stride + epw - 1;
    double* yw = ylds + cw * RW;
    uint32_t C[DE];
    double V[DE];
    auto load = [&](uint32_t p, int i) {
      const uint32_t k = min(min(lane, epw - 1) + p * stride, last);
      C[i] = ald_u32_nt(cu + k);
      V[i] = ald_f64_nt(vu + k);
    };
#pragma unroll
    for (int i = 0; i < DE; ++i) load(i, i);
    const uint32_t padded = (npan + DE - 1) / DE * DE;
    for (uint32_t b = 0; b < padded; b += DE) {
#pragma unroll
      for (int i = 0; i < DE; ++i) {
        const uint32_t p = b + i;
        vm_wait<2 * (DE - 1)>();  // slot i landed, DE - 1 panels of entries still in flight
        if (p < npan) {
          const uint32_t need = WL * (p / NS + 1);
          while (lds_ld(&landed[p % NS]) < need) __builtin_amdgcn_s_sleep(1);
          if (lane < epw) {
            const uint32_t c = C[i];
            const uint32_t row = ((c >> 16) * RW) >> 16;
            yw[row] = yw[row] + V[i] * xr[p % NS][(c & 0xFFFF) % P];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) lds_add(&consumed[p % NS], 1);
        }
        load(p + DE, i);
      }
    }
    vm_wait<0>();
  }
  __syncthreads();
  if (t == 0) out[u] = ylds[5] + ylds[R - 1];
}

// ---- G: x gathered from global memory (L1/L2), y block in LDS, all waves compute
template <int R, int P, int D, int DE>
__global__ __launch_bounds__(kT) void k_gather(const uint32_t* __restrict__ code, const double* __restrict__ vals,
                                               const double* __restrict__ x, double* __restrict__ out,
                                               uint32_t part_cols, int S, uint32_t epw) {
  constexpr int WC = kNW;
  constexpr uint32_t RW = R / WC;
  __shared__ double ylds[R];
  __shared__ uint32_t done[64];
  const int t = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const uint32_t u = blockIdx.x, h = (u / 8) % (uint32_t)S;
  const double* xp = x + (size_t)h * part_cols;
  const uint32_t npan = part_cols / P;
  for (uint32_t i = t; i < R; i += kT) ylds[i] = 0.0;
  if (t < 64) done[t] = 0;
  __syncthreads();
  const size_t ubase = (size_t)u * npan * WC * epw;
  const uint32_t* cu = code + ubase + w * epw;
  const double* vu = vals + ubase + w * epw;
  const uint32_t stride = WC * epw;
  const uint32_t last = (npan - 1) * stride + epw - 1;
  double* yw = ylds + w * RW;
  // per step p: gather x for p + 1 (its code landed), entries of p + DE, wait
  // for the gather of p, apply p.  The loop starts at p = -DE with dummy
  // gathers so every wait count is the steady-state one.
  static_assert(DE % 2 == 0 && DE >= 4, "ring");
  uint32_t C[DE];
  double V[DE], X[2];
  auto load = [&](int p, int i) {
    const uint32_t k = min(min(lane, epw - 1) + (uint32_t)max(p, 0) * stride, last);
    C[i] = ald_u32_nt(cu + k);
    V[i] = ald_f64_nt(vu + k);
  };
  auto gather = [&](int p, uint32_t c, int slot) {
    const size_t col = p >= 0 ? min((size_t)p * P + (c & 0xFFFF) % P, (size_t)part_cols - 1) : 0;
    X[slot] = ald_f64(xp + col);
  };
  const int padded = (int)((npan + DE - 1) / DE * DE);
  for (int b = -DE; b < padded; b += DE) {
#pragma unroll
    for (int i = 0; i < DE; ++i) {
      const int p = b + i;
      vm_wait<3 * (DE - 2)>();  // the code of p + 1 landed
      gather(p + 1, C[(i + 1) % DE], (i + 1) & 1);
      load(p + DE, i);
      vm_wait<5>();  // the gather of p landed
      if (p >= 0 && p < (int)npan) {
        if (D > 0 && p >= D) {
          while (lds_ld(&done[(p - D) & 63]) < (uint32_t)WC) __builtin_amdgcn_s_sleep(1);
        }
        if (lane < epw) {
          const uint32_t c = C[i];
          const uint32_t row = ((c >> 16) * RW) >> 16;
          yw[row] = yw[row] + V[i] * X[i & 1];
        }
        if (D > 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) {
            lds_add(&done[p & 63], 1);
            if (p >= 32) done[(p - 32) & 63] = 0;  // recycle (every wave has passed p - 32 + D)
          }
        }
      }
    }
  }
  vm_wait<0>();
  __syncthreads();
  if (t == 0) out[u] = ylds[5] + ylds[R - 1];
}

template <typename F>
static void timeit(const char* name, F launch, double ebytes, double xbytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  std::printf("%-44s %8.2f us  entries %6.0f GB/s  x %6.0f GB/s\n", name, us, ebytes / us / 1e3, xbytes / us / 1e3);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const std::string only = argc > 1 ? argv[1] : "";
  auto want = [&](const char* k) { return only.empty() || only.find(k) != std::string::npos; };
  const uint32_t U = 256;
  const size_t n = (size_t)U * kNE + (1 << 20);  // slack: layouts with a per-wave EPW pad
  uint32_t* code;
  double *vals, *x, *out;
  CK(hipMalloc(&code, 4 * n));
  CK(hipMalloc(&vals, 8 * n));
  CK(hipMalloc(&x, 8ull * kCols + 4096));
  CK(hipMalloc(&out, 8ull * U));
  {
    std::vector<uint32_t> hc(n);
    uint64_t z = 88172645463325252ull;
    for (size_t i = 0; i < n; ++i) {
      z ^= z << 13, z ^= z >> 7, z ^= z << 17;
      hc[i] = (uint32_t)(z >> 32);
    }
    CK(hipMemcpy(code, hc.data(), 4 * n, hipMemcpyHostToDevice));
  }
  CK(hipMemset(vals, 0, 8 * n));
  CK(hipMemset(x, 0, 8ull * kCols + 4096));
  const double eb = 12.0 * U * kNE;
  for (int rnd = 0; rnd < 2; ++rnd) {
    std::printf("-- round %d\n", rnd);
    for (int S : {3, 4}) {
      const uint32_t pc = kCols / S;
      const double xb = 8.0 * U * pc;
      char nm[96];
      if (want("E") && S == 3) {
        timeit("E 16 waves", [&] { hipLaunchKernelGGL((k_free<true, false, 0, 4000>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, 0);
        timeit("E 13 waves", [&] { hipLaunchKernelGGL((k_free<true, false, 3, 4000>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, 0);
      }
      if (want("X")) {
        std::snprintf(nm, sizeof nm, "X S=%d WL=3 P=4000", S);
        timeit(nm, [&] { hipLaunchKernelGGL((k_free<false, true, 3, 4000>), U, kT, 0, 0, code, vals, x, out, pc, S); }, 0, xb);
        std::snprintf(nm, sizeof nm, "EX free S=%d WL=3 P=4000", S);
        timeit(nm, [&] { hipLaunchKernelGGL((k_free<true, true, 3, 4000>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
      }
      if (want("A")) {
        if (S == 3) {  // R 12352: ring of 4 x 1920 columns (60 KiB)
          constexpr int P = 1920;
          const uint32_t npan = pc / P, epw = (kNE + npan * 13 - 1) / (npan * 13);
          std::snprintf(nm, sizeof nm, "A S=3 R=12352 NS=4 P=%d L=2 epw=%u", P, epw);
          timeit(nm, [&] { hipLaunchKernelGGL((k_async<12352, 4, P, 3, 2, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw); }, eb, xb);
          std::snprintf(nm, sizeof nm, "A S=3 R=12352 NS=4 P=%d L=1", P);
          timeit(nm, [&] { hipLaunchKernelGGL((k_async<12352, 4, P, 3, 1, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw); }, eb, xb);
        } else {  // R 16384: ring of 4 x 992 columns (31 KiB)
          constexpr int P = 992;
          const uint32_t npan = pc / P, epw = (kNE + npan * 13 - 1) / (npan * 13);
          std::snprintf(nm, sizeof nm, "A S=4 R=16384 NS=4 P=%d L=2 epw=%u", P, epw);
          timeit(nm, [&] { hipLaunchKernelGGL((k_async<16384, 4, P, 3, 2, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw); }, eb, xb);
          const uint32_t epw2 = (kNE + npan * 14 - 1) / (npan * 14);
          std::snprintf(nm, sizeof nm, "A S=4 R=16384 NS=4 P=%d L=2 WL=2", P);
          timeit(nm, [&] { hipLaunchKernelGGL((k_async<16384, 4, P, 2, 2, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw2); }, eb, xb);
        }
      }
      if (want("G") && S == 4) {
        constexpr int P = 2048;
        const uint32_t npan = pc / P, epw = (kNE + npan * 16 - 1) / (npan * 16);
        std::snprintf(nm, sizeof nm, "G S=4 R=16384 P=%d D=0 epw=%u", P, epw);
        timeit(nm, [&] { hipLaunchKernelGGL((k_gather<16384, P, 0, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw); }, eb, xb);
        timeit("G S=4 R=16384 P=2048 D=2", [&] { hipLaunchKernelGGL((k_gather<16384, P, 2, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw); }, eb, xb);
        constexpr int P2 = 1024;
        const uint32_t npan2 = pc / P2, epw2 = (kNE + npan2 * 16 - 1) / (npan2 * 16);
        timeit("G S=4 R=16384 P=1024 D=2", [&] { hipLaunchKernelGGL((k_gather<16384, P2, 2, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw2); }, eb, xb);
        constexpr int P3 = 4096;
        const uint32_t npan3 = pc / P3, epw3 = (kNE + npan3 * 16 - 1) / (npan3 * 16);
        if (epw3 <= 64)
          timeit("G S=4 R=16384 P=4096 D=1", [&] { hipLaunchKernelGGL((k_gather<16384, P3, 1, 8>), U, kT, 0, 0, code, vals, x, out, pc, S, epw3); }, eb, xb);
      }
    }
  }
  return 0;
}
