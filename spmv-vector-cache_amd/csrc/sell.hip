// k_sell: SELL-C-sigma SpMV for gfx950 -- one lane per row, ORDERED for any
// matrix.
//
// The vector-cache kernels need x to be streamed through LDS by every row
// block, which pays only while the matrix is dense enough per x element
// (choose_kernel); k_csr_lane, the ordered fallback, reads each row's entries
// with per-lane strides (no coalescing).  Here every row is still summed by
// ONE lane in ascending column order (SoftwareSpMV.cpp:59-64: products
// rounded, then added in order), but the entries are stored slice-major, so
// the 64 lanes of a wave read 64 consecutive 4-B column ids and 64
// consecutive 8-B values per step:
//
//   slice s: 256 rows (lane l owns rows l, l+64, l+128, l+192 -- four
//            independent chains per lane), width = its longest row; entry k
//            of sub-slice j, lane l at off[s] + (4k + j)*64 + l.
//   rows sorted by length inside windows of kSellSigma rows, so a slice's
//   rows have similar lengths (little padding); padded steps are loaded
//   (column 0, value 0: branch-free, coalesced) but never added.
//   hub rows (> kSellHub entries) -- over the CSR copy, entries loaded 256
//   at a time two stages ahead: ORDERED f64 gives each hub row one wave that
//   sums the products in one sequential chain through v_readlane (the order
//   is the contract); FAST / u64 cuts hub rows into pieces of <= 4096
//   entries, one wave each (four lane partials + a fixed xor tree), and the
//   last piece to finish adds the piece partials in piece order
//   (deterministic).
//
// Bytes per launch: 12 B per entry (padding included) + 8 B per slice row
// (row id, length) + 8 B per row of y written; x gathered from L2/MALL.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"

namespace hipspmv {
namespace {

constexpr int kHubG = 4;                    // chunks of 64 entries per hub pipeline stage
constexpr uint32_t kHubStage = 64 * kHubG;  // entries per stage

template <typename T>
__device__ __forceinline__ T nt(const T* p) {
  return __builtin_nontemporal_load(p);
}

// v as held by lane l (l wave-uniform)
template <typename T>
__device__ __forceinline__ T lane_value(T v, uint32_t l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), (int)l);
  return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
}

template <typename T>
__device__ __forceinline__ T xor_shuffle(T v, int m) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)u, m);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(u >> 32), m);
  return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
}

// The n >= 1 entries [base, base + n) of one row, the whole wave.  EXACT: the
// products added one after another to `acc` (the row's sequential chain; the
// result is wave-uniform).  Otherwise: four lane partials, then a fixed xor
// tree (every lane returns the same total; `acc` unused).
template <typename T, bool EXACT>
__device__ __forceinline__ T hub_entries(const SellArgs& a, uint32_t base, uint32_t n, T acc, int lane) {
#pragma clang fp contract(off)
  const T* __restrict__ vals = static_cast<const T*>(a.csr_vals);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  // entries of the stage starting at g0, indices clamped into the range (the
  // clamped copies are loaded but never consumed)
  auto load = [&](uint32_t g0, uint32_t* c, T* v) {
#pragma unroll
    for (int j = 0; j < kHubG; ++j) {
      const uint32_t e = min(g0 + (uint32_t)(j * 64 + lane), n - 1);
      c[j] = nt(a.colind + base + e);
      v[j] = nt(vals + base + e);
    }
  };
  uint32_t cA[kHubG];
  T vA[kHubG], p[kHubG], xs[kHubG];
  load(0, cA, vA);
#pragma unroll
  for (int j = 0; j < kHubG; ++j) xs[j] = x[cA[j]];
#pragma unroll
  for (int j = 0; j < kHubG; ++j) p[j] = vA[j] * xs[j];  // stage 0 products (rounded)
  load(kHubStage, cA, vA);                              // stage 1 entries
  T part[kHubG];
#pragma unroll
  for (int j = 0; j < kHubG; ++j) part[j] = T(0);
  for (uint32_t g0 = 0; g0 < n; g0 += kHubStage) {
    // gathers of the next stage and entries of the one after, in flight
    // while this stage's products are summed
#pragma unroll
    for (int j = 0; j < kHubG; ++j) xs[j] = x[cA[j]];
    uint32_t cB[kHubG];
    T vB[kHubG];
    load(g0 + 2 * kHubStage, cB, vB);
    const uint32_t m = min(kHubStage, n - g0);
    if (EXACT) {
      if (m == kHubStage) {
#pragma unroll
        for (int j = 0; j < kHubG; ++j) {
#pragma unroll
          for (int l = 0; l < 64; ++l) acc = acc + lane_value(p[j], (uint32_t)l);
        }
      } else {  // the last stage
#pragma unroll
        for (int j = 0; j < kHubG; ++j) {
          const uint32_t mj = m > (uint32_t)j * 64 ? min(64u, m - (uint32_t)j * 64) : 0u;
          for (uint32_t l = 0; l < mj; ++l) acc = acc + lane_value(p[j], l);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < kHubG; ++j)
        if (g0 + (uint32_t)(j * 64 + lane) < n) part[j] = part[j] + p[j];
    }
#pragma unroll
    for (int j = 0; j < kHubG; ++j) {
      p[j] = vA[j] * xs[j];
      cA[j] = cB[j];
      vA[j] = vB[j];
    }
  }
  if (EXACT) return acc;
  T s = (part[0] + part[1]) + (part[2] + part[3]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s = s + xor_shuffle(s, d);  // every lane: the same total
  return s;
}

// v rotated one lane up the wave: lane l receives lane l-1's value, lane 0
// lane 63's (DPP wave_ror:1, two 32-bit moves)
template <typename T>
__device__ __forceinline__ T wave_ror1(T v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x13C, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x13C, 0xF, 0xF, false);
  return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
}

// ORDERED f64: hub row r in one wave, one chain from y_in (or +0.0) --
// SoftwareSpMV's own sequence of rounded adds, so it cannot be split; what
// can be made short is each link.  A stage holds 64 * kChainG consecutive
// entries, lane l the kChainG entries l*kChainG.. in its registers, their
// products formed by every lane at once (invalid ones -0.0, which leaves
// every sum unchanged).  The chain then visits the lanes in order: every
// lane adds its products to `acc`, and a wave rotation hands the sum of
// lane l to lane l+1 (lane 63's to lane 0, for the next stage), so only
// lane l's sum is the chain's at step l.  Per entry one dependent add plus a
// share of the rotation: chain_probe measured a register-fed add chain at
// 4.3 cycles per add, and the v_readlane chain this replaces at 20.6.
// Entries two stages ahead and gathers one stage ahead stay in flight.
template <typename T, int G>
__device__ __forceinline__ void hub_row_exact(const SellArgs& a, uint32_t w, int lane) {
#pragma clang fp contract(off)
  constexpr uint32_t S = 64 * G;
  const T* __restrict__ vals = static_cast<const T*>(a.csr_vals);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const uint32_t r = a.hubs[w], base = a.rowptr[r], n = a.rowptr[r + 1] - base;
  // the chain is latency-bound: the longest hub rows (w: longest first) get
  // first call on their SIMD's issue slots, over shorter chains and slices
  if (w < 4)
    __builtin_amdgcn_s_setprio(3);
  else if (w < 64)
    __builtin_amdgcn_s_setprio(2);
  else
    __builtin_amdgcn_s_setprio(1);
  auto load = [&](uint32_t g0, uint32_t* c, T* v) {  // clamped: the copies past the row are never added
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t e = min(g0 + (uint32_t)lane * G + j, n - 1);
      c[j] = nt(a.colind + base + e);
      v[j] = nt(vals + base + e);
    }
  };
  auto products = [&](uint32_t g0, const T* v, const T* xs, T* p) {
#pragma unroll
    for (int j = 0; j < G; ++j) p[j] = g0 + (uint32_t)lane * G + j < n ? v[j] * xs[j] : T(-0.0);
  };
  uint32_t cA[G], cB[G];
  T vA[G], vB[G], xs[G], p[G];
  load(0, cA, vA);
#pragma unroll
  for (int j = 0; j < G; ++j) xs[j] = x[cA[j]];
  products(0, vA, xs, p);
  load(S, cA, vA);
  T acc = a.beta ? static_cast<const T*>(a.y_in)[r] : T(0);  // lane 0's is the chain's
  for (uint32_t g0 = 0; g0 < n; g0 += S) {
#pragma unroll
    for (int j = 0; j < G; ++j) xs[j] = x[cA[j]];  // next stage's gathers
    load(g0 + 2 * S, cB, vB);                      // and the entries of the one after
    // the chain touches no memory: keep the scheduler from moving the loads'
    // consumers (and their waits) into it
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int l = 0; l < 64; ++l) {
      T s = acc;
#pragma unroll
      for (int j = 0; j < G; ++j) s = s + p[j];
      acc = wave_ror1(s);
    }
    __builtin_amdgcn_sched_barrier(0);
    products(g0 + S, vA, xs, p);  // waits for the gathers only (the entry loads are younger)
#pragma unroll
    for (int j = 0; j < G; ++j) {
      cA[j] = cB[j];
      vA[j] = vB[j];
    }
  }
  if (lane == 0) static_cast<T*>(a.y_out)[r] = acc;
}

// hub_row_exact with the gathers two stages ahead (experimental): at stage k
// the products of k are in p, the gathers of k+1 have been in flight since
// stage k-1, and the gathers of k+2 and the entries of k+3 are issued before
// k's chain -- two chains of latency cover each gather.  Buffers rotate with
// period 3 (unrolled, so no register copy waits on a load in flight).  The
// adds are hub_row_exact's, in the same order: the same bits.
template <typename T, int G>
__device__ __forceinline__ void hub_row_exact2(const SellArgs& a, uint32_t w, int lane) {
#pragma clang fp contract(off)
  constexpr uint32_t S = 64 * G;
  const T* __restrict__ vals = static_cast<const T*>(a.csr_vals);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const uint32_t r = a.hubs[w], base = a.rowptr[r], n = a.rowptr[r + 1] - base;
  if (w < 4)
    __builtin_amdgcn_s_setprio(3);
  else if (w < 64)
    __builtin_amdgcn_s_setprio(2);
  else
    __builtin_amdgcn_s_setprio(1);
  uint32_t c[3][G];
  T v[3][G], xs[3][G], p[G];
  auto load = [&](uint32_t g0, uint32_t* cc, T* vv) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t e = min(g0 + (uint32_t)lane * G + j, n - 1);
      cc[j] = nt(a.colind + base + e);
      vv[j] = nt(vals + base + e);
    }
  };
  auto gather = [&](const uint32_t* cc, T* xx) {
#pragma unroll
    for (int j = 0; j < G; ++j) xx[j] = x[cc[j]];
  };
  auto products = [&](uint32_t g0, const T* vv, const T* xx) {
#pragma unroll
    for (int j = 0; j < G; ++j) p[j] = g0 + (uint32_t)lane * G + j < n ? vv[j] * xx[j] : T(-0.0);
  };
  load(0, c[0], v[0]);
  load(S, c[1], v[1]);
  gather(c[0], xs[0]);
  products(0, v[0], xs[0]);
  gather(c[1], xs[1]);
  load(2 * S, c[2], v[2]);
  T acc = a.beta ? static_cast<const T*>(a.y_in)[r] : T(0);
  auto stage = [&](auto I, uint32_t g0) {
    constexpr int i = decltype(I)::value, i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    gather(c[i2], xs[i2]);   // stage k+2's gathers
    load(g0 + 3 * S, c[i], v[i]);  // stage k+3's entries (buffer i is free: p holds stage k)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int l = 0; l < 64; ++l) {
      T s = acc;
#pragma unroll
      for (int j = 0; j < G; ++j) s = s + p[j];
      acc = wave_ror1(s);
    }
    __builtin_amdgcn_sched_barrier(0);
    products(g0 + S, v[i1], xs[i1]);  // waits for stage k+1's gathers only
  };
  for (uint32_t g0 = 0; g0 < n; g0 += 3 * S) {
    stage(std::integral_constant<int, 0>{}, g0);
    if (g0 + S >= n) break;
    stage(std::integral_constant<int, 1>{}, g0 + S);
    if (g0 + 2 * S >= n) break;
    stage(std::integral_constant<int, 2>{}, g0 + 2 * S);
  }
  if (lane == 0) static_cast<T*>(a.y_out)[r] = acc;
}

// FAST / u64: one piece of a hub row.  A row in several pieces is finished by
// the wave whose ticket add returns np - 1: it adds the piece partials in
// piece order.  Hand-off as in k_vcache's split combine (MI355X_MICROARCH.md,
// "Valid forms" row 1): agent-scope (sc1) store of the partial, vmcnt(0),
// agent-scope ticket add; the last arriver reads the partials with
// agent-scope loads and resets the ticket for the next launch.
template <typename T>
__device__ __forceinline__ void hub_piece(const SellArgs& a, uint32_t pid, int lane) {
#pragma clang fp contract(off)
  const uint32_t* pc = a.pieces + (size_t)pid * kSellPieceWords;
  const uint32_t r = pc[0], begin = pc[1], n = pc[2], idx = pc[3], np = pc[4], tk = pc[5];
  const T s = hub_entries<T, false>(a, a.rowptr[r] + begin, n, T(0), lane);
  if (lane != 0) return;
  T* y = static_cast<T*>(a.y_out);
  if (np == 1) {
    y[r] = a.beta ? static_cast<const T*>(a.y_in)[r] + s : s;
    return;
  }
  uint64_t* parts = static_cast<uint64_t*>(a.partial) + (pid - idx);
  __hip_atomic_store(parts + idx, __builtin_bit_cast(uint64_t, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t old = __hip_atomic_fetch_add(a.tickets + tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old != np - 1) return;
  __hip_atomic_store(a.tickets + tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  T t = __builtin_bit_cast(T, __hip_atomic_load(parts, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (uint32_t q = 1; q < np; ++q)
    t = t + __builtin_bit_cast(T, __hip_atomic_load(parts + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  y[r] = a.beta ? static_cast<const T*>(a.y_in)[r] + t : t;
}

// One slice s: lane `lane` sums rows row[s][j*64 + lane], j = 0..3.  NTL:
// the slice's entries load non-temporally (the slices s >= nt_from), so the
// others and x stay in L2 / the Infinity Cache.
template <typename T, bool NTL>
__device__ __forceinline__ void slice_rows(const SellArgs& a, uint32_t s, int lane) {
#pragma clang fp contract(off)
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const uint64_t off = a.off[s];
  const uint32_t width = a.width[s];
  uint32_t r[4], n[4];
  T acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t i = (size_t)s * kSellRows + j * 64 + lane;
    r[j] = a.row[i];
    n[j] = a.len[i];
    acc[j] = a.beta && r[j] != kSellNoRow ? static_cast<const T*>(a.y_in)[r[j]] : T(0);
  }
  const uint32_t* __restrict__ c = a.col + off + lane;
  const T* __restrict__ v = static_cast<const T*>(a.vals) + off + lane;
  auto ld = [](const auto* p) {
    if constexpr (NTL)
      return nt(p);
    else
      return *p;
  };
  // Software pipeline over pairs of steps (8 entries per lane), two register
  // buffers A/B: gathers of one pair are issued, then the entries of the
  // pair after it, then the products wait for the gathers only (vmcnt counts
  // in issue order, so the younger entry loads stay in flight).  Clamped
  // indices keep every prefetch inside the slice.
  auto load2 = [&](uint32_t k0, uint32_t* cc, T* vv) {
    const size_t i0 = (size_t)k0 * 4 * 64;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      cc[q] = ld(c + i0 + q * 64);
      vv[q] = ld(v + i0 + q * 64);
    }
    // compiler-only barriers (emit nothing): without a possible memory write
    // after these loads, InstCombine folds a loop-carried load into one load
    // at the loop header (the prefetch is lost); the scheduling barrier keeps
    // the machine scheduler from interleaving the three groups (gathers, next
    // entries, products), which would put a wait for a young load in front
    // of older work
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto add2 = [&](uint32_t k0, const T* xx, const T* vv) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = q & 3;
      const T t = madd(acc[j], vv[q], xx[q]);
      acc[j] = k0 + (q >> 2) < n[j] ? t : acc[j];
    }
  };
  auto gather2 = [&](const uint32_t* cc, T* xx) {
    __builtin_amdgcn_sched_barrier(0);  // after the previous products
#pragma unroll
    for (int q = 0; q < 8; ++q) xx[q] = x[cc[q]];
    asm volatile("" ::: "memory");  // the gathers issue before the next entry loads
    __builtin_amdgcn_sched_barrier(0);
  };
  uint32_t k = 0;
  if (width >= 4) {
    uint32_t cA[8], cB[8];
    T vA[8], vB[8], xx[8];
    load2(0, cA, vA);
    for (; k + 4 <= width; k += 4) {
      gather2(cA, xx);
      load2(k + 2, cB, vB);
      add2(k, xx, vA);
      gather2(cB, xx);
      load2(min(k + 4, width - 2), cA, vA);
      add2(k + 2, xx, vB);
    }
  }
  for (; k < width; ++k) {  // the last 0-3 steps
    const size_t i0 = (size_t)k * 4 * 64;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T t = madd(acc[j], ld(v + i0 + j * 64), x[ld(c + i0 + j * 64)]);
      acc[j] = k < n[j] ? t : acc[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (r[j] != kSellNoRow) static_cast<T*>(a.y_out)[r[j]] = acc[j];
}

// Waves [0, H) take the hub work -- EXACT: the hub rows (longest first), one
// wave each, G entries per lane per chain stage; otherwise the hub-row pieces
// -- and the rest one slice each.
template <typename T, bool EXACT, int G, int D = 1>
__device__ __forceinline__ void sell_wave(const SellArgs& a) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * 4 + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t H = EXACT ? a.nhubs : a.npieces;
  if (w < H) {
    if (EXACT) {
      if constexpr (D == 2)
        hub_row_exact2<T, G>(a, w, lane);
      else
        hub_row_exact<T, G>(a, w, lane);
    }
    else
      hub_piece<T>(a, w, lane);
    return;
  }
  const uint32_t s = w - H;
  if (s < a.nslices) {
    if (s >= a.nt_from)
      slice_rows<T, true>(a, s, lane);
    else
      slice_rows<T, false>(a, s, lane);
  }
}

template <typename T, bool EXACT>
__global__ __launch_bounds__(256) void k_sell(const SellArgs a) {
  sell_wave<T, EXACT, kChainG>(a);
}
// experimental (option "sell_chain_g"): the ORDERED hub chain with G entries
// per lane per stage -- the same adds in the same order, so the same bits
template <int G, int D>
__global__ __launch_bounds__(256) void k_sell_chain(const SellArgs a) {
  sell_wave<double, true, G, D>(a);
}

template <typename T, bool EXACT>
hipError_t launch(const SellArgs& a, hipStream_t s) {
  const uint64_t waves = (uint64_t)(EXACT ? a.nhubs : a.npieces) + a.nslices;
  if (waves == 0) return hipSuccess;
  const dim3 grid((uint32_t)((waves + 3) / 4));
  if constexpr (EXACT) {
    // option sell_chain = 10 * G + D (G entries per lane per stage, gathers D stages ahead)
    switch (a.chain_g) {
      case 82: hipLaunchKernelGGL((k_sell_chain<8, 2>), grid, dim3(256), 0, s, a); return hipGetLastError();
      case 121: hipLaunchKernelGGL((k_sell_chain<12, 1>), grid, dim3(256), 0, s, a); return hipGetLastError();
      case 122: hipLaunchKernelGGL((k_sell_chain<12, 2>), grid, dim3(256), 0, s, a); return hipGetLastError();
      case 161: hipLaunchKernelGGL((k_sell_chain<16, 1>), grid, dim3(256), 0, s, a); return hipGetLastError();
      default: break;
    }
  }
  hipLaunchKernelGGL((k_sell<T, EXACT>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_sell(int dtype, const SellArgs& a, hipStream_t s) {
  if (dtype == HIPSPMV_U64) return launch<uint64_t, false>(a, s);  // integer sums: order-free
  return a.exact ? launch<double, true>(a, s) : launch<double, false>(a, s);
}

}  // namespace hipspmv
