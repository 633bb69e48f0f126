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
// the same wait, tying the registers it makes valid: the compiler cannot
// read them before it, nor hand their registers to another value while the
// loads may still write them (an asm-load result it thought dead was reused
// while the load was in flight: the round-4 probe's GPU fault)
template <typename R>
__device__ __forceinline__ void tie(R& r) {  // volatile asms keep their order: a tie after a wait stays after it
  asm volatile("" : "+v"(r));
}
template <int N, typename... R>
__device__ __forceinline__ void vm_wait_tie(R&... r) {
  vm_wait<N>();
  (tie(r), ...);
}

// ---- E / X / EX: free-running roles
// MAP 1: unit u's column part is (u mod 8) mod S, so with S = 4 each XCD
// (round-robin dispatch: u mod 8) streams one 2 MiB part (its L2 holds it).
// C11: the entry stream as 11-byte entries (u16 column, u8 row step, f64 value).
template <bool E, bool X, int WL, int P, int MAP = 0, bool C11 = false>
__global__ __launch_bounds__(kT) void k_free(const uint32_t* __restrict__ code, const double* __restrict__ vals,
                                             const double* __restrict__ x, double* __restrict__ out,
                                             uint32_t part_cols, int S) {
  __shared__ double xb[2][P];
  __shared__ double pad[12000];  // one workgroup per CU, as the product
  constexpr int WC = kNW - WL, CT = WC * 64, EPT = 2, DE = 4;
  const int t = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const uint32_t u = blockIdx.x, h = MAP ? (u & 7) % (uint32_t)S : (u / 8) % (uint32_t)S;
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
    const uint16_t* cu16 = reinterpret_cast<const uint16_t*>(code) + (size_t)u * kNE;
    const uint8_t* du8 = reinterpret_cast<const uint8_t*>(code) + (size_t)kNE * 256 * 2 + (size_t)u * kNE;
    auto load = [&](uint32_t s, uint32_t* c, double* v) {
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const uint32_t i = min(s * STEP + j * CT + ct, kNE - 1);
        if (C11)
          c[j] = (uint32_t)__builtin_nontemporal_load(cu16 + i) | (uint32_t)__builtin_nontemporal_load(du8 + i) << 16;
        else
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

// ---- EW: the entry stream with 16-byte loads (each lane four consecutive
// entries: one dwordx4 of codes, two of values), free-running, beside the
// free-running x loaders (X) of k_free
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <bool X, int WL, int P, int MAP, int DE>
__global__ __launch_bounds__(kT) void k_wide(const uint32_t* __restrict__ code, const double* __restrict__ vals,
                                             const double* __restrict__ x, double* __restrict__ out,
                                             uint32_t part_cols, int S) {
  __shared__ double xb[2][P];
  __shared__ double pad[12000];
  constexpr int WC = kNW - WL, CT = WC * 64;
  const int t = threadIdx.x;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  const uint32_t u = blockIdx.x, h = MAP ? (u & 7) % (uint32_t)S : (u / 8) % (uint32_t)S;
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
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ND) : "memory");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    const int ct = t - WL * 64;
    const uint32_t* cu = code + (size_t)u * kNE;
    const double* vu = vals + (size_t)u * kNE;
    constexpr uint32_t STEP = 4 * CT;  // entries per step
    constexpr uint32_t NSTEPS = (kNE + STEP - 1) / STEP;
    u32x4v C[DE];
    double V[DE][4];
    auto load = [&](uint32_t s, int i) {
      const uint32_t e = min(s * STEP + 4 * ct, kNE - 4);  // 4 consecutive entries, 16-B aligned
      C[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(cu + e));
      const u32x4v v0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(vu + e));
      const u32x4v v1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(vu + e + 2));
      V[i][0] = __builtin_bit_cast(double, (uint64_t)v0.x | (uint64_t)v0.y << 32);
      V[i][1] = __builtin_bit_cast(double, (uint64_t)v0.z | (uint64_t)v0.w << 32);
      V[i][2] = __builtin_bit_cast(double, (uint64_t)v1.x | (uint64_t)v1.y << 32);
      V[i][3] = __builtin_bit_cast(double, (uint64_t)v1.z | (uint64_t)v1.w << 32);
    };
#pragma unroll
    for (int d = 0; d < DE; ++d) load(d, d);
    constexpr uint32_t PADDED = (NSTEPS + DE - 1) / DE * DE;
    for (uint32_t b = 0; b < PADDED; b += DE) {
#pragma unroll
      for (int i = 0; i < DE; ++i) {
        acc += (double)C[i].x * V[i][0] + (double)C[i].y * V[i][1] + (double)C[i].z * V[i][2] +
               (double)C[i].w * V[i][3];
        load(b + i + DE, i);
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
  static_assert(DE == 8, "ring (the final wait ties 8 slots)");
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
        vm_wait_tie<2 * (DE - 1)>(C[i], V[i]);  // slot i landed, DE - 1 panels of entries still in flight
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
    vm_wait_tie<0>(C[0], C[1], C[2], C[3], C[4], C[5], C[6], C[7], V[0], V[1], V[2], V[3], V[4], V[5], V[6], V[7]);
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
  static_assert(DE == 8, "ring (the final wait ties 8 slots)");
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
  // fully unrolled (S = 4 parts: npan = 2^18 / P panels, a constant): no loop
  // back-edge, so no phi copy of a ring register whose load is in flight
  constexpr int NPAN = (int)((kCols / 4) / P), PADDED = (NPAN + DE - 1) / DE * DE;
#pragma unroll
  for (int b = -DE; b < PADDED; b += DE) {
#pragma unroll
    for (int i = 0; i < DE; ++i) {
      const int p = b + i;
      vm_wait_tie<3 * (DE - 2)>(C[(i + 1) % DE]);  // the code of p + 1 landed
      gather(p + 1, C[(i + 1) % DE], (i + 1) & 1);
      vm_wait_tie<2>(C[i], V[i]);  // entries of p landed (older than the gather of p + 1)
      const uint32_t c = C[i];  // slot i is reloaded next
      const double v = V[i];
      load(p + DE, i);
      vm_wait_tie<5>(X[i & 1]);  // the gather of p landed
      if (p >= 0 && p < NPAN) {
        if (D > 0 && p >= D) {
          while (lds_ld(&done[(p - D) & 63]) < (uint32_t)WC) __builtin_amdgcn_s_sleep(1);
        }
        if (lane < epw) {
          const uint32_t row = ((c >> 16) * RW) >> 16;
          yw[row] = yw[row] + v * X[i & 1];
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
  vm_wait_tie<0>(C[0], C[1], C[2], C[3], C[4], C[5], C[6], C[7], V[0], V[1], V[2], V[3], V[4], V[5], V[6], V[7],
                 X[0], X[1]);
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
      if (want("M") && S == 4) {
        timeit("X S=4 WL=3 P=4000 XCD map", [&] { hipLaunchKernelGGL((k_free<false, true, 3, 4000, 1>), U, kT, 0, 0, code, vals, x, out, pc, S); }, 0, xb);
        timeit("EX free S=4 WL=3 P=4000 XCD map", [&] { hipLaunchKernelGGL((k_free<true, true, 3, 4000, 1>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
        timeit("E 13 waves, 11-byte entries", [&] { hipLaunchKernelGGL((k_free<true, false, 3, 4000, 0, true>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, 0);
        timeit("EX free S=4 XCD map, 11-byte entries", [&] { hipLaunchKernelGGL((k_free<true, true, 3, 4000, 1, true>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
      }
      if (want("W")) {
        std::snprintf(nm, sizeof nm, "E 13 waves, 16-B loads (DE=3)");
        timeit(nm, [&] { hipLaunchKernelGGL((k_wide<false, 3, 4000, 1, 3>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, 0);
        std::snprintf(nm, sizeof nm, "EX free S=%d XCD map, 16-B entry loads (DE=3)", S);
        timeit(nm, [&] { hipLaunchKernelGGL((k_wide<true, 3, 4000, 1, 3>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
        std::snprintf(nm, sizeof nm, "EX free S=%d XCD map, 16-B entry loads (DE=2)", S);
        timeit(nm, [&] { hipLaunchKernelGGL((k_wide<true, 3, 4000, 1, 2>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
        std::snprintf(nm, sizeof nm, "EX free S=%d, 16-B entry loads (DE=3)", S);
        timeit(nm, [&] { hipLaunchKernelGGL((k_wide<true, 3, 4000, 0, 3>), U, kT, 0, 0, code, vals, x, out, pc, S); }, eb, xb);
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
