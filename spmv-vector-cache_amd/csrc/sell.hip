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

// ORDERED f64, a hub row of at least kSellIso entries in a 1024-thread
// workgroup of its own (k_sell_iso).  A wave64 f64 add issues over 4 cycles
// of its SIMD, so a chain sharing its SIMD with other busy waves runs at a
// fraction of its rate (C5 shard 0: the longest row alone 864 µs, among the
// other hub waves 1478 µs).  Here wave 0 runs the chain and nothing else;
// the helper waves -- all 15 others when G is a multiple of 15 (the product,
// kIsoG = 45), else the 12 off the chain's SIMD while waves 4, 8, 12 only
// meet the barriers -- load the entries NB stages ahead, gather x two stages
// ahead and write stage i's products to an LDS ring.  Lane l of the chain
// owns products l*G..l*G+G-1 of a stage (slot j*65 + l: conflict-free reads,
// and the padding spreads the helpers' writes over the banks) and the lanes
// hand the sum on by DPP rotation, as hub_row_exact does: the same adds, in
// the same order, so the same bits.  At most 20 waves of this kernel fit a
// CU, so a 1024-thread workgroup keeps its CU to itself.
template <typename T, int G>
__device__ __forceinline__ void hub_row_isolated(const SellArgs& a, uint32_t hub) {
#pragma clang fp contract(off)
  constexpr int GA = 2;
  constexpr uint32_t S = 64 * G;                  // products per stage
  // helper threads: waves off the chain's SIMD (768), or with G a multiple
  // of 15 (experimental) every wave but the chain (960)
  constexpr bool ALL = G % 15 == 0;
  constexpr uint32_t NH = ALL ? 960u : 768u;
  constexpr int PPT = (S + NH - 1) / NH;          // products per helper thread
  constexpr int NB = PPT >= 3 ? 3 : 4;            // entry buffers: loads NB stages ahead
  constexpr uint32_t RS = 65;                     // ring row stride: lane l's j-th product at j*65 + l
  __shared__ T ring[2][RS * G];
  const T* __restrict__ vals = static_cast<const T*>(a.csr_vals);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t r = a.hubs[hub], base = a.rowptr[r], n = a.rowptr[r + 1] - base;
  const uint32_t nst = (n + S - 1) / S;
  // LDS writes done, then the barrier; global loads stay in flight across it
  auto barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  if (wv == 0) {  // ---- the chain: stage i - 1 in iteration i
    __builtin_amdgcn_s_setprio(3);
    T acc = a.beta ? static_cast<const T*>(a.y_in)[r] : T(0);
    barrier();  // iteration 0: the helpers produce stage 0
    for (uint32_t i = 1; i <= nst; ++i) {
      const T* slot = ring[(i - 1) & 1];
      T p[G];
#pragma unroll
      for (int j = 0; j < G; ++j) p[j] = slot[j * RS + lane];
#pragma unroll
      for (int l = 0; l < 64; ++l) {
        T s = acc;
#pragma unroll
        for (int j = 0; j < G; ++j) s = s + p[j];
        acc = wave_ror1(s);
      }
      barrier();
    }
    if (lane == 0) static_cast<T*>(a.y_out)[r] = acc;
    return;
  }
  if (!ALL && (wv & 3) == 0) {  // ---- the chain's SIMD: barriers only
    for (uint32_t i = 0; i <= nst; ++i) barrier();
    return;
  }
  // ---- helpers: thread ht makes products ht, ht + NH, ... (< S) of every stage
  const uint32_t ht = (uint32_t)(ALL ? wv - 1 : wv - (wv >> 2) - 1) * 64 + lane;  // -> [0, NH)
  uint32_t c[NB][PPT];
  T v[NB][PPT], xg[NB][PPT];
  auto load = [&](uint32_t st, int k) {  // clamped: copies past the row are never used
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const uint32_t e = min(st * S + min(ht + NH * q, S - 1), n - 1);
      c[k][q] = nt(a.colind + base + e);
      v[k][q] = nt(vals + base + e);
    }
  };
  auto gather = [&](int k) {
#pragma unroll
    for (int q = 0; q < PPT; ++q) xg[k][q] = x[c[k][q]];
  };
#pragma unroll
  for (int k = 0; k < NB; ++k) load(k, k);
#pragma unroll
  for (int k = 0; k < GA; ++k) gather(k);
  asm volatile("" ::: "memory");
  auto iter = [&](auto K, uint32_t i) {
    constexpr int k = decltype(K)::value, kg = (k + GA) % NB;
    // stage i: the products (or -0.0 past the row, which leaves every sum as
    // it is) into the slot of chain lane e / G, position e % G
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const uint32_t e = ht + NH * q;
      if (q == 0 || e < S) ring[i & 1][(e % G) * RS + e / G] = i * S + e < n ? v[k][q] * xg[k][q] : T(-0.0);
    }
    gather(kg);       // stage i + GA's gathers
    load(i + NB, k);  // stage i + NB's entries
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    barrier();
  };
  uint32_t i = 0;
  for (; i + NB <= nst; i += NB) {
    iter(std::integral_constant<int, 0>{}, i);
    iter(std::integral_constant<int, 1>{}, i + 1);
    iter(std::integral_constant<int, 2>{}, i + 2);
    if constexpr (NB == 4) iter(std::integral_constant<int, NB - 1>{}, i + 3);
  }
  // the last 0..NB-1 stages (unrolled roles continue from i % NB == 0), then
  // the chain's last iteration's barrier
  if (i < nst) iter(std::integral_constant<int, 0>{}, i++);
  if (i < nst) iter(std::integral_constant<int, 1>{}, i++);
  if constexpr (NB == 4)
    if (i < nst) iter(std::integral_constant<int, 2>{}, i++);
  barrier();
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
template <typename T, bool EXACT, int G>
__device__ __forceinline__ void sell_wave(const SellArgs& a) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * 4 + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t H = EXACT ? a.nhubs : a.npieces;
  if (w < H) {
    if (EXACT)
      hub_row_exact<T, G>(a, w, lane);
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
// ORDERED f64 when some hub row has at least kSellIso entries: those rows
// isolated (hub_row_isolated), the rest as k_sell does them, in 1024-thread
// workgroups
// Blocks: [0, niso) the isolated rows; then the slices, 4 a block (waves
// 4-15 exit at once, so a block's slices spread over as many CUs as k_sell's
// 256-thread blocks do: 16 latency-bound slices on one CU ran 3.7x slower);
// then the other hub rows, 16 waves (rows) a block.  The slices go before
// the hub blocks: dispatched after them, their long-latency waves started
// only once the ~1000 hub blocks had drained and ended the launch.
template <int G>
__global__ __launch_bounds__(1024) void k_sell_iso(const SellArgs a) {
  if (blockIdx.x < a.niso) {
    hub_row_isolated<double, G>(a, blockIdx.x);
    return;
  }
  const int lane = threadIdx.x & 63;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t H = a.nhubs - a.niso, sb = (a.nslices + 3) / 4, b = blockIdx.x - a.niso;
  if (b < sb) {
    if (wv >= 4) return;
    const uint32_t s = b * 4 + wv;
    if (s < a.nslices) {
      if (s >= a.nt_from)
        slice_rows<double, true>(a, s, lane);
      else
        slice_rows<double, false>(a, s, lane);
    }
    return;
  }
  const uint32_t w = (b - sb) * 16 + wv;
  if (w < H) hub_row_exact<double, kChainG>(a, a.niso + w, lane);
}

template <typename T, bool EXACT>
hipError_t launch(const SellArgs& a, hipStream_t s) {
  const uint64_t waves = (uint64_t)(EXACT ? a.nhubs : a.npieces) + a.nslices;
  if (waves == 0) return hipSuccess;
  const dim3 grid((uint32_t)((waves + 3) / 4));
  if constexpr (EXACT) {
    // isolated chains when some hub row is long enough (option sell_chain 1: never;
    // 2, 3 (experimental): stages of G = 12 (12 helper waves) or 30)
    if (a.niso > 0 && a.chain_g != 1) {
      const dim3 g((uint32_t)(a.niso + (a.nhubs - a.niso + 15) / 16 + (a.nslices + 3) / 4));
      if (a.chain_g == 2)
        hipLaunchKernelGGL(k_sell_iso<12>, g, dim3(1024), 0, s, a);
      else if (a.chain_g == 3)
        hipLaunchKernelGGL(k_sell_iso<30>, g, dim3(1024), 0, s, a);
      else
        hipLaunchKernelGGL(k_sell_iso<kIsoG>, g, dim3(1024), 0, s, a);
      return hipGetLastError();
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
