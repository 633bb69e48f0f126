// k_vcache: the LDS "vector cache" SpMV kernel for gfx950.
//
// The reference's accelerators stream A in column order and keep the output
// vector y in an on-chip vector cache (chisel/cache-new/NoWMVectorCache.scala,
// chisel/frontend/SpMVFrontendNewCache.scala:102-151).  Here one 1024-thread
// workgroup owns a block of rows: their y accumulators live in LDS for the
// whole launch, and x is streamed through LDS in panels of VP columns, so every
// x gather and every y update is an LDS access; HBM sees each nonzero once.
//
// Work unit = (row block b, column part h).  SPLIT == 1 (ordered geometry):
// one part, every row's products are added in ascending column order, starting
// from y_in or +0.0 -- bit-identical to SoftwareSpMV.  SPLIT == 3 (product
// FAST geometry) or 4 (experimental): three (four) column parts per block,
// each streaming a third (quarter) of x -- the x requests hold each CU's
// L1->L2 slots -- combined in fixed order y = p0 + p1 + p2
// (+ p3) by whichever workgroup of the block finishes last: deterministic,
// FAST-mode tolerance.
//
// Waves are specialised (producer/consumer): waves [0, WL) stream x panels
// into LDS (LD == 0: register-staged, two panels ahead; LD == 1: LDS-DMA,
// global_load_lds_dwordx4 straight into the next slot, one panel ahead);
// waves [WL, 16) stream the unit's entries (DE panels ahead) and apply them.
// Each role waits only on its own vmcnt, so the L2-served x stream and the
// HBM-served entry stream overlap; one workgroup barrier per panel hands the
// next x panel over.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "combine.h"
#include "device_common.h"
#include "vc_map.h"
#include "hipspmv_internal.h"
#include "kernels.h"

namespace hipspmv {

// lane l gets lane l + 1's value inside its 16-lane row (DPP row_shl:1; lane
// 15 of a row gets 0): the first step of a run continuation when the layout
// keeps every run inside one row (CX == 5)
__device__ __forceinline__ uint32_t dpp_next32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false);
}
template <typename T>
__device__ __forceinline__ T dpp_next(T v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(T, (uint64_t)dpp_next32((uint32_t)u) | (uint64_t)dpp_next32((uint32_t)(u >> 32)) << 32);
}

// Per-geometry configuration.  LDS: VR*8 + 2*VP*8 + kVcSegMax*4 = 163840 B.
template <int SPLIT>
struct VcCfg;
template <>
struct VcCfg<1> {  // 4096 rows; x panel 63.5 KiB; 8 loader waves (8 pairs/lane), 8 compute waves
  // (round 2: 2 / 5 LDS-DMA loaders with 14 / 11 compute waves and cross-lane runs measured 247 / 201 us
  // against 217 here -- each CU streams all 8 MB of x, so the loaders bound it; AUTO's ORDERED kernel is sell)
  static constexpr int VR = kVcOrdered.rows, VP = kVcOrdered.panel, WL = 8, DE = 4, EPT = 3;
};
static_assert(VcCfg<1>::WL == (int)kVcOrderedLoaders, "build_xmask's words are the ordered loader waves'");
template <>
struct VcCfg<3> {  // 12352 rows; x panel 31.25 KiB; 3 LDS-DMA loader waves, 13 compute waves (2 entries/lane)
  // round-2 sweep on C3 (WL, DE, EPT, loader): 3/4/2 DMA 124.6 us; 3/4/3 DMA 131.2; 2/4/2 DMA 125.8-126.3;
  // 2/6/2 DMA 126.8; 2/8/2 DMA 127.0;
  // 4/4/3 DMA 128.9; 6/4/3 DMA 129.7; 6/4/3 registers 131.6; 4/4/3, 5/4/3, 6/6/3 registers 133.6-134.2;
  // 2/4/3 DMA 132.4; 8/4/4 registers 150.4; 1/4/2 and 1/6/2 DMA 172-173 (one loader wave falls behind)
  static constexpr int VR = kVcSplit.rows, VP = kVcSplit.panel, WL = 3, DE = 4, EPT = 2;
};
template <>
struct VcCfg<4> {  // 16384 rows; x panel 15.5 KiB; 2 loader waves (8 pairs/lane), 14 compute waves
  static constexpr int VR = kVcSplit4.rows, VP = kVcSplit4.panel, WL = 2, DE = 4, EPT = 2;
};

// AB: ablation mask for the diagnostic build (tools/vc_ablate.hip); the
// product instantiates AB = 0 and every hook folds away.  Bits: 1 no x loads,
// 2 no x LDS stores, 4 no entry loads, 8 no compute, 16 x always from panel 0,
// 32 no per-panel barrier, 64 no column-part combine (wrong results, timing only),
// 128 profile stamps, results unchanged (option "profile"): 8 u32
// per workgroup at tickets + 4 * nblocks + 8 * blockIdx.x (SPLIT 1: at partial):
// s_memrealtime (100 MHz) at start, main-loop start, main-loop end, exit; the
// combine ticket; s_memtime cycles summed over the steps: loader wave 0 working,
// loader wave 0 waiting at the step barrier, first compute wave waiting there.
// 256 / 512 / 1024 / 2048 / 4096: the entries of row blocks b >= nblocks/2,
// 5/8, 3/8, 1/4, 1/8 loaded
// non-temporally (Infinity-Cache residency experiment).
// 16384 (xlane 3 path): y updated by one LDS atomic add per owner (the same
// one update per row and step; deterministic).
// 8192 (with 64; diagnostic, tools/step_trace.hip): step trace -- lane 0 of every
// wave stores {ready, arrive, release, applied} (s_memtime low words: its data
// landed, it reached the step barrier, the barrier let it go, its LDS apply
// retired -- compute waves) of every step, as uint4
// at partial + 16 * ((blockIdx.x * 16 + wave) * 256 + step); step slot 255: {kernel
// entry, 0, release of the prologue barrier}.
template <typename T, int SPLIT, int WL = VcCfg<SPLIT>::WL, int DE = VcCfg<SPLIT>::DE, int EPT = VcCfg<SPLIT>::EPT,
          int AB = 0, int MAP = 0, bool NT = false, int LD = 0, int CX = 0>
__global__ __launch_bounds__(kVcThreads) void k_vcache(const uint32_t* __restrict__ seg,
                                                        const uint32_t* __restrict__ ecode,
                                                        const T* __restrict__ evals, const T* __restrict__ x,
                                                        const T* __restrict__ y_in, T* __restrict__ y_out,
                                                        T* __restrict__ partial, uint32_t* __restrict__ tickets,
                                                        uint32_t rows, uint32_t cols, uint32_t rows_per_block,
                                                        uint32_t nblocks, uint32_t npanels, uint32_t part_panels,
                                                        uint32_t npad, uint32_t last, int beta,
                                                        uint32_t nt_from, const uint64_t* __restrict__ xmask) {
#pragma clang fp contract(off)
  constexpr int VR = VcCfg<SPLIT>::VR, VP = VcCfg<SPLIT>::VP;
  constexpr int VT = kVcThreads, NW = VT / 64, WC = NW - WL;
  constexpr int LT = WL * 64, CT = WC * 64;  // loader / compute lanes
  constexpr uint32_t PAIRS = VP / 2;         // 16-byte pairs per panel
  constexpr int NJ = (PAIRS + LT - 1) / LT;  // pairs per loader lane per panel
  static_assert(VR * 8 + 2 * VP * 8 + kVcSegMax * 4 <= 163840, "LDS budget");
  static_assert(WL > 0 && WC > 0, "both roles need waves");
  static_assert(SPLIT == 1 || SPLIT == 3 || SPLIT == 4, "column parts");
  __shared__ alignas(16) T ylds[VR];  // 16-B aligned: the combine moves row pairs
  __shared__ T xb[2][VP];
  __shared__ uint32_t segl[kVcSegMax];

  const int t = threadIdx.x;
  const bool loader = __builtin_amdgcn_readfirstlane(t >> 6) < WL;  // wave-uniform role
  uint32_t b = blockIdx.x, h = 0;
  if (MAP == 1 && SPLIT > 1 && vc_map1_applies<SPLIT>(nblocks)) {
    vc_unit_map1<SPLIT>(blockIdx.x, b, h);  // XCD-aware placement (csrc/vc_map.h)
  } else if (MAP == 2 && SPLIT > 1) {
    vc_unit_map2(blockIdx.x, nblocks * SPLIT, nblocks, b, h);  // one column part per XCD where it can
  } else if (SPLIT > 1) {  // unit i -> (b, h): the parts of a block are 8 dispatch slots apart (vc_unit_map0)
    const uint32_t g = blockIdx.x / (8 * SPLIT), rem = blockIdx.x % (8 * SPLIT);
    const uint32_t nbg = min(8u, nblocks - g * 8);
    h = rem / nbg;
    b = g * 8 + rem % nbg;
  }
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry (workgroup-uniform, before any barrier)
  const uint32_t nr = min(rows_per_block, rows - r0);
  uint32_t* const sbuf = (SPLIT == 1 ? reinterpret_cast<uint32_t*>(partial) : tickets + 4 * nblocks) + 8 * blockIdx.x;
  auto stamp = [&](int k, uint32_t v) {
    if ((AB & 128) && t == 0) sbuf[k] = v;
  };
  auto now = [] { return (uint32_t)__builtin_amdgcn_s_memrealtime(); };
  if (AB & 128) stamp(0, now());
  const uint32_t p0 = vc_part_first(h, npanels, SPLIT);             // first global panel of this unit
  const uint32_t npu = vc_part_first(h + 1, npanels, SPLIT) - p0;   // >= 1 (vcache_grid_ok)
  const uint32_t* sp = seg + ((size_t)b * SPLIT + h) * (npad + 1);
  if ((uint32_t)t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = (beta && h == 0) ? y_in[r0 + i] : T(0);

  // ---- loader role: x panels, branch-free 16-byte loads clamped to the last
  // in-bounds pair; for odd cols the final element is patched from a scalar
  // load by the lane owning its LDS slot.
  const uint32_t cmax = (cols - 2) & ~1u;
  const T xlast = x[cols - 1];
  const uint32_t wl = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  // xmask (SPLIT 1, register-staged loaders): bit 8 j + k of word [unit][panel][loader wave wl] says
  // whether the unit's entries of that panel use x line wl * 8 + j * LT / 8 + k (build_xmask,
  // csrc/plan.cpp) -- the 128-byte line that lanes 8 k .. 8 k + 7 of the wave's j-th load cover; the
  // lanes of a line no entry uses load nothing (no L2 request), and their LDS slots are never read
  constexpr bool XMASK = SPLIT == 1 && LD == 0 && NJ * 8 <= 64;  // one 64-bit word per loader wave and panel
  // the mask word of panel s (all ones without a mask); the LD 0 loader loads it a step before its
  // x loads need it (LD 2's counted vmcnt waits assume every load issued: no mask there)
  auto mask_of = [&](uint32_t s) -> uint64_t {
    return (XMASK && xmask) ? xmask[((size_t)b * npanels + p0 + min(s, npu - 1)) * WL + wl] : ~0ull;
  };
  const __amdgpu_buffer_rsrc_t xrs = buf_rsrc(x, XMASK ? cols * (uint32_t)sizeof(T) : 0u);
  auto load_x = [&](uint32_t s, u64x2* r, uint64_t m = ~0ull) {
    if (AB & 1) return;
    const uint32_t base = (AB & 16) ? 0 : (p0 + min(s, npu - 1)) * VP;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const uint32_t ci = min(base + 2 * (t + j * LT), cmax);
      if constexpr (XMASK) {
        // branch-free: a lane of an unused line gets an out-of-range offset in the descriptor of x --
        // zero, and no memory request (a divergent `if` around a plain load made hipcc wait vmcnt(0)
        // before every load of the ring)
        const bool need = (m >> (j * 8 + (lane >> 3))) & 1u;
        r[j] = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(
                                             xrs, need ? (int)(ci * (uint32_t)sizeof(T)) : (int)0x80000000, 0, 0));
      } else {
        const T* src = x + ci;
        r[j] = LD == 2 ? ald_128(src) : *reinterpret_cast<const u64x2*>(src);
      }
    }
  };
  // LD == 1: the loader lanes' 16-byte chunks go straight into LDS.  A
  // wave-instruction writes 64 consecutive chunks (wave-uniform base + lane *
  // 16 B); chunk c of a panel is issued by wave (c / 64) % WL in its
  // instruction c / (64 * WL), lanes past the panel's end masked off.
  constexpr int NDMA = (PAIRS + LT - 1) / LT;
  auto dma_x = [&](uint32_t s) {
    if (AB & 1) return;
    const uint32_t base = (AB & 16) ? 0 : (p0 + min(s, npu - 1)) * VP;
    T* slot = xb[s & 1];
#pragma unroll
    for (int j = 0; j < NDMA; ++j) {
      const uint32_t c0 = (j * WL + wl) * 64;  // first chunk of this wave-instruction
      if (c0 + lane < PAIRS)
        __builtin_amdgcn_global_load_lds(
            (const void*)(x + min(base + 2 * (c0 + lane), cmax)),
            (__attribute__((address_space(3))) void*)(slot + 2 * c0), 16, 0, 0);
    }
  };
  auto patch_x = [&](uint32_t s) {  // odd cols: the last element, after this wave's DMA landed
    if ((cols & 1) && p0 + s == npanels - 1) {
      const uint32_t sl = cols - 1 - (p0 + s) * VP, c = sl >> 1;
      if (c < PAIRS && ((c / 64) % WL) == wl && (c & 63) == lane) xb[s & 1][sl] = xlast;
    }
  };
  auto store_x = [&](uint32_t s, const u64x2* r) {
    if (AB & 2) return;
    T* dst = xb[s & 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if ((j + 1) * LT <= (int)PAIRS || (uint32_t)(t + j * LT) < PAIRS)
        *reinterpret_cast<u64x2*>(&dst[2 * (t + j * LT)]) = r[j];
    if ((cols & 1) && p0 + s == npanels - 1) {
      const uint32_t slot = cols - 1 - (p0 + s) * VP;
      if ((uint32_t)t == (slot >> 1) % LT) dst[slot] = xlast;
    }
  };

  // ---- compute role: entries at clamped indices (branch-free), validity
  // checked at use.  A row run's first entry is held by one lane; its
  // continuation entries (MORE) are read back from memory (rare: several
  // entries of one row inside one panel).
  const int ct = t - LT;
  // beg_in: the step's first entry when the caller has it (CX 5), else read here
  auto load_e = [&](uint32_t s, uint32_t* c, T* v, auto ntc, uint32_t beg_in = ~0u) {
    if (AB & 4) {
#pragma unroll
      for (int j = 0; j < EPT; ++j) c[j] = kVcCont;
      return;
    }
    const uint32_t beg = beg_in != ~0u ? beg_in : segl[min(s, npad)];
    if constexpr (CX == 4 || CX == 6) {
      // masked: a lane past the step's segment gets an out-of-range offset in
      // a descriptor of the unit's entries -- zero, and no memory request
      // (clamped lanes re-read the next segment: 1.1x the entry requests here,
      // 1.68x at four parts)
      const uint32_t e0 = __builtin_amdgcn_readfirstlane(segl[0]);
      const uint32_t ne = __builtin_amdgcn_readfirstlane(segl[npu]) - e0;
      const uint32_t end = segl[min(s + 1, npad)] - e0;
      const __amdgpu_buffer_rsrc_t dc = buf_rsrc(ecode + e0, 4 * ne), dv = buf_rsrc(evals + e0, 8 * ne);
      constexpr int aux = decltype(ntc)::value || NT ? 2 : 0;  // nt
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const uint32_t q = beg - e0 + ct + j * CT;
        const bool in = q < end;
        c[j] = __builtin_amdgcn_raw_buffer_load_b32(dc, in ? (int)(4 * q) : (int)0x80000000, 0, aux);
        v[j] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(dv, in ? (int)(8 * q) : (int)0x80000000, 0, aux));
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t i = min(beg + ct + j * CT, last);
      if (CX == 2) {
        c[j] = ald_u32(ecode + i);
        v[j] = ald_64(evals + i);
      } else if (NT || decltype(ntc)::value) {  // non-temporal: kept out of the Infinity Cache
        c[j] = __builtin_nontemporal_load(ecode + i);
        v[j] = __builtin_nontemporal_load(evals + i);
      } else {
        c[j] = ecode[i];
        v[j] = evals[i];
      }
    }
  };
  auto run = [&](uint32_t i, uint32_t code, T v, const T* xs) {
    const uint32_t row = (code >> 16) & 0x3FFF;
    T acc = madd(ylds[row], v, xs[code & 0xFFFF]);
    while (code & kVcMore) {
      ++i;
      code = ecode[i];
      acc = madd(acc, evals[i], xs[code & 0xFFFF]);
    }
    ylds[row] = acc;
  };
  // A row has one run per step (its entries of a panel are consecutive in the
  // segment), so the run heads of a step name distinct rows: every slot's x and
  // y reads issue before any y write (the compiler cannot prove the rows
  // distinct and would chain slot j + 1's reads behind slot j's write), the
  // same additions in the same order.
  auto apply = [&](uint32_t s, const uint32_t* c, const T* v) {
    if (AB & 8) return;
    const T* xs = xb[s & 1];
    const uint32_t beg = segl[s], end = segl[s + 1];
    T acc[EPT];
    bool head[EPT];
    // CX 6: a slot no lane of this wave holds an entry of (wave-uniform) issues none of its LDS reads
    // (the ordered geometry's 512 lanes x 3 slots hold ~1000 entries per step: the third is empty)
    const uint32_t wq0 = __builtin_amdgcn_readfirstlane(beg + (ct & ~63u));
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t q = beg + ct + j * CT;
      head[j] = q < end && !(c[j] & kVcCont);
      if (CX == 6 && wq0 + j * CT >= end) {
        acc[j] = T(0);
        continue;
      }
      const uint32_t row = (c[j] >> 16) & 0x3FFF;
      const T xv = xs[head[j] ? (c[j] & 0xFFFF) : 0u], yv = ylds[head[j] ? row : 0u];
      acc[j] = madd(yv, v[j], xv);
    }
    if constexpr (CX == 6) {
      // the layout keeps every run inside its 16-lane row (place_segments_banked): a run head takes its
      // first continuation entry from the next lane by DPP (every lane executes the DPP), and re-reads
      // from memory only from the third entry of a run on (C3: runs of two, 24 % of the steps)
      uint32_t cn[EPT];
      T vn[EPT], xn[EPT];
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        cn[j] = dpp_next32(c[j]);
        vn[j] = dpp_next(v[j]);
      }
#pragma unroll
      for (int j = 0; j < EPT; ++j) xn[j] = xs[head[j] && (c[j] & kVcMore) ? (cn[j] & 0xFFFF) : 0u];
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        if (head[j] && (c[j] & kVcMore)) {
          acc[j] = madd(acc[j], vn[j], xn[j]);
          uint32_t i = beg + ct + j * CT + 1, code = cn[j];
          while (code & kVcMore) {  // runs of three or more
            ++i;
            code = ecode[i];
            acc[j] = madd(acc[j], evals[i], xs[code & 0xFFFF]);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        if (head[j] && (c[j] & kVcMore)) {  // run continuation, re-read from memory (rare)
          uint32_t i = beg + ct + j * CT, code = c[j];
          while (code & kVcMore) {
            ++i;
            code = ecode[i];
            acc[j] = madd(acc[j], evals[i], xs[code & 0xFFFF]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      if (head[j]) ylds[(c[j] >> 16) & 0x3FFF] = acc[j];
    for (uint32_t q = beg + EPT * CT + ct; q < end; q += CT) {  // beyond the register window (slow path)
      const uint32_t code = ecode[q];
      if (!(code & kVcCont)) run(q, code, evals[q], xs);
    }
  };

  // CX == 1: the same arithmetic with no vector-memory access besides the
  // entry ring, so every wave's vmcnt waits stay partial and the DE-deep
  // prefetch survives (a run continuation or overflow load is the youngest
  // VMEM op and its wait drains the whole ring: measured round 1, see
  // DESIGN.md §6.5).  Every valid lane forms its product; a run head adds its
  // continuation products taken from the next lanes of its wave
  // (__shfl_down: LDS crossbar, lgkmcnt); a run that continues past the wave
  // (lane 63 -> next wave) finishes with scalar loads.  Requires every segment
  // to fit the register window (max_seg <= EPT*CT, checked at launch).
  const uint32_t lw = t & 63;
  auto sload32 = [](const uint32_t* p) {
    uint32_t r;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
    return r;
  };
  auto sload64 = [](const T* p) {
    uint64_t r;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
    return __builtin_bit_cast(T, r);
  };
  auto apply_cx = [&](uint32_t s, const uint32_t* c, const T* v) {
    if (AB & 8) return;
    const T* xs = xb[s & 1];
    const uint32_t beg = segl[s], end = segl[s + 1];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t q = beg + ct + j * CT;
      const uint32_t code = c[j];
      const bool valid = q < end;
      const T p = valid ? v[j] * xs[code & 0xFFFF] : T(0);  // rounded product (contract off)
      const bool own = valid && !(code & kVcCont);
      const uint32_t row = (code >> 16) & 0x3FFF;
      T acc = own ? ((AB & 16384) ? p : ylds[row] + p) : T(0);
      bool more = own && (code & kVcMore);
      bool fb = false;
      uint32_t fbi = 0;
      uint32_t k0 = 1;
      if constexpr (CX == 5) {  // the layout keeps each run inside its 16-lane row: step 1 by DPP, no LDS
        const T p1 = dpp_next(p);
        const uint32_t c1 = dpp_next32(code);
        if (more) {
          acc = acc + p1;
          more = (c1 & kVcMore) != 0;
        }
        k0 = 2;
      }
      for (uint32_t k = k0; __builtin_amdgcn_ballot_w64(more) != 0; ++k) {  // wave-uniform trip count
        const T pk = __shfl_down(p, k);
        const uint32_t ck = __shfl_down(code, k);
        if (more) {
          if (lw + k < 64) {
            acc = acc + pk;
            more = (ck & kVcMore) != 0;
          } else {  // the run continues in the next wave's lanes
            fb = true;
            fbi = q + k;
            more = false;
          }
        }
      }
      for (uint64_t m = __builtin_amdgcn_ballot_w64(fb); m; m &= m - 1) {  // rare
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        uint32_t i = __builtin_amdgcn_readlane(fbi, l);
        const uint64_t ab = __builtin_bit_cast(uint64_t, acc);
        T a = __builtin_bit_cast(T, (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)ab, l) |
                                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(ab >> 32), l) << 32));
        uint32_t cd;
        do {
          cd = sload32(ecode + i);
          const T pv = sload64(evals + i) * xs[cd & 0xFFFF];
          a = a + pv;
          ++i;
        } while (cd & kVcMore);
        if (lw == l) acc = a;
      }
      if (own) {
        if (AB & 16384)  // one LDS atomic (ds_add_f64 / ds_add_u64) instead of the read and the write
          __hip_atomic_fetch_add(&ylds[row], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
          ylds[row] = acc;
      }
    }
  };

  // CX == 5 (a layout whose runs stay inside 16-lane rows, place_segments_banked):
  // the same arithmetic as CX 1-3 without branches around the LDS accesses --
  // both slots' x and y reads issue together, then one wait (CX 3 waited for
  // the x read, then the y read, per slot: four round trips per step) -- and
  // the step's segment bounds come from registers (beg, end) instead of LDS.
  // A run head takes its first continuation from the next lane by DPP, longer
  // runs by shuffles as in CX 1-3; no run leaves its row, so none leaves the wave.
  auto apply5 = [&](uint32_t s, const uint32_t* c, const T* v, uint32_t beg, uint32_t end) {
    if (AB & 8) return;
    const T* xs = xb[s & 1];
    T xv[EPT], yv[EPT], p[EPT], acc[EPT];
    uint32_t row[EPT];
    bool own[EPT], more[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      row[j] = (c[j] >> 16) & 0x3FFF;
      xv[j] = xs[c[j] & 0xFFFF];  // unconditional: every lane's code is a clamped entry, in range
      yv[j] = ylds[row[j]];
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const bool valid = beg + ct + j * CT < end;
      p[j] = valid ? v[j] * xv[j] : T(0);  // rounded product (contract off)
      own[j] = valid && !(c[j] & kVcCont);
      acc[j] = own[j] ? yv[j] + p[j] : T(0);
      more[j] = own[j] && (c[j] & kVcMore);
      const T p1 = dpp_next(p[j]);
      const uint32_t c1 = dpp_next32(c[j]);
      if (more[j]) {
        acc[j] = acc[j] + p1;
        more[j] = (c1 & kVcMore) != 0;
      }
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      for (uint32_t k = 2; __builtin_amdgcn_ballot_w64(more[j]) != 0; ++k) {  // runs of 3+ (rare)
        const T pk = __shfl_down(p[j], k);
        const uint32_t ck = __shfl_down(c[j], k);
        if (more[j]) {
          acc[j] = acc[j] + pk;
          more[j] = (ck & kVcMore) != 0;
        }
      }
      if (own[j]) ylds[row[j]] = acc[j];
    }
  };

  // Each role runs its own loop with exactly one workgroup barrier per panel
  // (npu + 1 barriers in all, the same count in both), so the two register
  // rings are never live together and the allocator overlays them.
  auto barrier = [&]() {
    if (AB & 32) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  // profile (AB & 128): cycles between step barriers (work) and inside them (wait)
  uint64_t pf_work = 0, pf_wait = 0, pf_mark = 0;
  auto pbarrier = [&]() {
    if (AB & 128) {
      const uint64_t a = __builtin_amdgcn_s_memtime();
      pf_work += a - pf_mark;
      barrier();
      pf_mark = __builtin_amdgcn_s_memtime();
      pf_wait += pf_mark - a;
    } else {
      barrier();
    }
  };
  // step trace (AB & 8192): stamps, and the store after each step barrier
  auto tr_now = [] {
    asm volatile("" ::: "memory");
    const uint32_t v = (uint32_t)__builtin_amdgcn_s_memtime();
    asm volatile("" ::: "memory");
    return v;
  };
  const uint32_t t_entry = (AB & 8192) ? tr_now() : 0;
  auto tr_rel = [&](uint32_t s, uint32_t a, uint32_t b, uint32_t c = 0) {
    if (!(AB & 8192)) return;
    const uint32_t r = tr_now();
    if ((t & 63) == 0)
      reinterpret_cast<uint4*>(partial)[((size_t)blockIdx.x * 16 + (uint32_t)(t >> 6)) * 256 + min(s, 255u)] =
          make_uint4(a, b, r, c);
  };
  static_assert(!(AB & 8192) || (AB & 64), "the step trace lives in the partials: no combine");
  // CX >= 2: both roles run a step count padded to the unroll (extra steps do
  // no work but keep their loads and barrier), so no loop exits mid-group.
  // An early exit inside the unrolled group is what makes hipcc's waitcnt
  // pass merge a path with fewer loads in flight into the loop header and
  // emit vmcnt(0) there (tools/vmcnt_check.py finds the same infeasible
  // path); without it the compiler's own waits are exact (CX == 3).
  // (The ordered geometry, SPLIT 1 / CX 0, does not pad: its unpadded loader
  // loop drains the two-panel x ring before every odd step's stores, and
  // padding fixed that but cost its three extra steps and measured 2 % slower:
  // 171.9 against 168-170 us, profiles/r05/logs/ab_xmask_b_pad.log.)
  constexpr bool PAD = CX >= 2 && CX != 6;
  constexpr uint32_t ALIGN = (DE % 2 == 0) ? DE : 2 * DE;
  const uint32_t nsteps = PAD ? (npu + ALIGN - 1) / ALIGN * ALIGN : npu;
  __syncthreads();  // segl visible
  if (loader && LD == 1) {
    // panel s+1 is fetched into slot (s+1)&1 during step s; the slot was last
    // read in step s-1, which the previous barrier closed
    dma_x(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    patch_x(0);
    barrier();
    tr_rel(255, t_entry, 0);
    if (AB & 128) {
      stamp(1, now());
      pf_mark = __builtin_amdgcn_s_memtime();
    }
    for (uint32_t s = 0; s < nsteps; ++s) {
      if (s + 1 < npu) dma_x(s + 1);
      if constexpr (AB & 32768) {
        // ablation (wrong results, timing only): the loaders do not wait for their panel before the
        // step barrier -- the bound on what decoupling the x latency from the step could gain
        asm volatile("s_barrier" ::: "memory");
        continue;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t_ready = (AB & 8192) ? tr_now() : 0;
      if (s + 1 < npu) patch_x(s + 1);
      pbarrier();
      tr_rel(s, t_ready, t_ready);
    }
    if constexpr (AB & 32768) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (loader && LD == 2) {
    // same ring, asm loads: storing x(s+1) waits for it with x(s+2)'s NJ
    // loads (issued one step later) still in flight
    u64x2 R[2][NJ];
    load_x(0, R[0]);
    vm_wait<0>();
    store_x(0, R[0]);
    load_x(1, R[1]);
    load_x(2, R[0]);
    barrier();
    for (uint32_t base = 0; base < nsteps; base += 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t s = base + i;
        if (!PAD && s >= npu) break;
        vm_wait<((AB & 1) || LD != 2) ? 0 : NJ>();  // (branch only live for LD == 2)
        if (s + 1 < npu) store_x(s + 1, R[(i + 1) & 1]);
        load_x(s + 3, R[(i + 1) & 1]);
        barrier();
      }
    }
    vm_wait<0>();
  } else if (loader) {
    u64x2 R[2][NJ];  // R[(s+1)&1] holds x(s+1) during step s
    load_x(0, R[0], mask_of(0));
    store_x(0, R[0]);
    load_x(1, R[1], mask_of(1));
    load_x(2, R[0], mask_of(2));
    uint64_t mnext = mask_of(3);  // panel s + 3's mask word, loaded during step s - 1
    barrier();
    tr_rel(255, t_entry, 0);
    if (AB & 128) {
      stamp(1, now());
      pf_mark = __builtin_amdgcn_s_memtime();
    }
    for (uint32_t base = 0; base < nsteps; base += 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t s = base + i;  // parity of s == parity of i
        if (!PAD && s >= npu) break;
        const uint64_t m3 = mnext;
        mnext = mask_of(s + 4);
        if (s + 1 < npu) store_x(s + 1, R[(i + 1) & 1]);
        const uint32_t t_ready = (AB & 8192) ? tr_now() : 0;  // panel s + 1 landed and stored
        load_x(s + 3, R[(i + 1) & 1], m3);
        const uint32_t t_arr = (AB & 8192) ? tr_now() : 0;
        pbarrier();
        tr_rel(s, t_ready, t_arr);
      }
    }
  } else {
    // the entry role; ntc: this unit's entries loaded non-temporally -- the
    // row blocks b >= nt_from (the AB bits 256-4096 fix the threshold instead):
    // nt entry lines leave L2 and the Infinity Cache to x and to the blocks
    // below the threshold, whose entries then stay resident across launches
    // 
    auto entries = [&](auto ntc) {
      uint32_t EC[DE][EPT];
      T EV[DE][EPT];
      if constexpr (CX == 5) {
        // segment bounds ride with the ring: SB/SE[i] of the step slot i holds
        uint32_t SB[DE], SE[DE];
#pragma unroll
        for (int i = 0; i < DE; ++i) {
          SB[i] = segl[min((uint32_t)i, npad)];
          SE[i] = segl[min((uint32_t)i + 1, npad)];
          load_e(i, EC[i], EV[i], ntc, SB[i]);
        }
        barrier();
        tr_rel(255, t_entry, 0);
        for (uint32_t base = 0; base < nsteps; base += DE) {
#pragma unroll
          for (int i = 0; i < DE; ++i) {
            const uint32_t s = base + i;
            // the bounds of step s + DE, read before the apply so their LDS latency hides behind it
            const uint32_t nb = segl[min(s + DE, npad)], ne = segl[min(s + DE + 1, npad)];
            uint32_t t_ready = 0, t_arr = 0, t_app = 0;
            if (AB & 8192) {
              vm_wait<1 + (2 * EPT + 1) * (DE - 1)>();
              t_ready = tr_now();
            }
            if (s < npu) apply5(s, EC[i], EV[i], SB[i], SE[i]);
            if (AB & 8192) {
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              t_app = tr_now();
            }
            SB[i] = nb;
            SE[i] = ne;
            load_e(s + DE, EC[i], EV[i], ntc, nb);
            if (AB & 8192) t_arr = tr_now();
            pbarrier();
            tr_rel(s, t_ready, t_arr, t_app);
          }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < DE; ++i) load_e(i, EC[i], EV[i], ntc);
      barrier();
      tr_rel(255, t_entry, 0);
      if (AB & 128) pf_mark = __builtin_amdgcn_s_memtime();
      for (uint32_t base = 0; base < nsteps; base += DE) {
#pragma unroll
        for (int i = 0; i < DE; ++i) {
          const uint32_t s = base + i;
          if (!PAD && s >= npu) break;
          if (CX == 2) vm_wait<(AB & 4) ? 0 : (DE - 1) * 2 * EPT>();  // slot i landed, DE-1 steps still in flight
          uint32_t t_ready = 0, t_arr = 0, t_app = 0;
          if (AB & 8192) {  // this step's entries landed: each later step issued 2 * EPT loads + 1 trace store
            vm_wait<1 + (2 * EPT + 1) * (DE - 1)>();
            t_ready = tr_now();
          }
          if (CX && CX != 6) {
            if (!PAD || s < npu) apply_cx(s, EC[i], EV[i]);
          } else {
            if (!PAD || s < npu) apply(s, EC[i], EV[i]);
          }
          if (AB & 8192) {  // the apply's LDS work retired, then the next loads issued
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            t_app = tr_now();
          }
          load_e(s + DE, EC[i], EV[i], ntc);
          if (AB & 8192) t_arr = tr_now();
          pbarrier();
          tr_rel(s, t_ready, t_arr, t_app);
        }
      }
      if (CX == 2) vm_wait<0>();  // the clamped prefetches past the last panel
    };
    constexpr int NTAB = AB & (256 | 512 | 1024 | 2048 | 4096);
    const uint32_t thr = NTAB == 0 ? nt_from
                       : (AB & 512) ? nblocks * 5 / 8 : (AB & 1024) ? nblocks * 3 / 8
                       : (AB & 2048) ? nblocks / 4 : (AB & 4096) ? nblocks / 8 : nblocks / 2;
    if (NT || b >= thr)
      entries(std::true_type{});
    else
      entries(std::false_type{});
  }
  if (AB & 128) {
    if (t == 0) {
      sbuf[5] = (uint32_t)pf_work;
      sbuf[6] = (uint32_t)pf_wait;
    }
    if (t == LT) sbuf[7] = (uint32_t)pf_wait;
    __syncthreads();
    stamp(2, now());
  }
  if (AB & 64) {  // ablation: no combine, y straight from LDS (timing only)
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
    if (AB & 128) stamp(3, now());
    return;
  }
  if (SPLIT == 1) {
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
    if (AB & 128) stamp(3, now());
    return;
  }
  // ---- combine the column parts, fixed order p0 + p1 + p2 (+ p3): unit h
  // owns share h of the block's row pairs (csrc/combine.h); counters at
  // tickets + 4 b, partials of part q of block b at partial + (q * nblocks + b) * VRP
  __syncthreads();  // segl is the combine's scratch from here
  owner_combine<T, SPLIT, VT, (VR + 1) & ~1u>(ylds, segl, partial, tickets + 4 * (size_t)b, b, h, nblocks, nr,
                                              y_out + r0, t);
  if (AB & 128) stamp(3, now());
}

template <typename T, int SPLIT, int LD, int CX = 0, int MAP = 0>
static void launch_one(const VcacheArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((k_vcache<T, SPLIT, VcCfg<SPLIT>::WL, VcCfg<SPLIT>::DE, VcCfg<SPLIT>::EPT, 0, MAP, false, LD, CX>),
                     dim3(a.nblocks * SPLIT), dim3(kVcThreads), 0, s, a.seg, a.code, (const T*)a.vals,
                     (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial, a.tickets, a.rows, a.cols,
                     a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.last, a.beta, a.nt_from,
                     a.xmask);
}

#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
// every form (make EXPERIMENTAL=1: lib/exp/libhipspmv.so, loaded under HIPSPMV_EXPERIMENTAL=1)
template <typename T, int SPLIT, int MAP = 0>
static void dispatch(const VcacheArgs& a, hipStream_t s, int ld, int cx) {
  if constexpr (SPLIT == 3) {  // three loader waves: LDS-DMA only (a register-staged panel would spill)
    if (cx == 0)
      launch_one<T, SPLIT, 1, 0, MAP>(a, s);
    else if (cx == 1)
      launch_one<T, SPLIT, 1, 1, MAP>(a, s);
    else if (cx == 2)
      launch_one<T, SPLIT, 1, 2, MAP>(a, s);
    else if (cx == 3)
      launch_one<T, SPLIT, 1, 3, MAP>(a, s);
    else if (cx == 5)
      launch_one<T, SPLIT, 1, 5, MAP>(a, s);
    else
      launch_one<T, SPLIT, 1, 4, MAP>(a, s);
  } else if (cx == 4) {  // (split 3 only)
    launch_one<T, SPLIT, 0, 3, MAP>(a, s);
  } else if (cx == 5) {  // (a banked layout: runs inside 16-lane rows)
    launch_one<T, SPLIT, 0, 5, MAP>(a, s);
  } else if (cx == 6) {  // the ordered geometry on a banked layout: CX 0 with the DPP first continuation
    ld == 1 ? launch_one<T, SPLIT, 1, 6, MAP>(a, s) : launch_one<T, SPLIT, 0, 6, MAP>(a, s);
  } else if (cx == 0) {
    ld == 1 ? launch_one<T, SPLIT, 1, 0, MAP>(a, s) : launch_one<T, SPLIT, 0, 0, MAP>(a, s);
  } else if (cx == 1) {
    ld == 1 ? launch_one<T, SPLIT, 1, 1, MAP>(a, s) : launch_one<T, SPLIT, 0, 1, MAP>(a, s);
  } else if (cx == 2) {
    ld == 1 ? launch_one<T, SPLIT, 1, 2, MAP>(a, s) : launch_one<T, SPLIT, 2, 2, MAP>(a, s);
  } else {
    ld == 1 ? launch_one<T, SPLIT, 1, 3, MAP>(a, s) : launch_one<T, SPLIT, 0, 3, MAP>(a, s);
  }
}
#endif

template <typename T>
hipError_t launch_vcache(const VcacheArgs& a, hipStream_t s) {
  // the layout's geometry must be the one the kernel is compiled for
  const VcGeom g = a.split == 1 ? kVcOrdered : a.split == 3 ? kVcSplit : kVcSplit4;
  if (!vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.panel,
                      a.split, g))
    return hipErrorInvalidValue;
  // cross-lane continuation needs every segment inside the register window
  auto window = [](int split) {
    const int wl = split == 1 ? VcCfg<1>::WL : split == 3 ? VcCfg<3>::WL : VcCfg<4>::WL;
    const int ept = split == 1 ? VcCfg<1>::EPT : split == 3 ? VcCfg<3>::EPT : VcCfg<4>::EPT;
    return (uint32_t)((kVcThreads / 64 - wl) * 64 * ept);
  };
  // xlane 1: cross-lane continuation; 2: also padded loops and asm rings
  // (entries, and x unless LDS-DMA stages it) with explicit vmcnt waits;
  // 3: cross-lane continuation and padded loops, the compiler's own waits;
  // 4 (split 3): 3 with the entry loads masked past each step's segment;
  // 5 (split 3, a layout whose runs stay inside 16-lane rows --
  // place_segments_banked): 3 with the first continuation step by DPP.
  // -1 (default): 5 for the split geometry where the layout allows it, else 3
  // (C3: 131.7 us against 135.7 with the run continuation re-read from
  // memory), 0 for the others.
  // 6 (ordered, a layout whose runs stay inside 16-lane rows): 0 with the
  // first continuation step by DPP.
  int xl = a.xlane < 0 ? (a.split >= 3 ? (a.row_runs ? 5 : 3) : 0) : a.xlane;
  if (xl == 5 && !a.row_runs) xl = 3;
  if (xl == 6 && (!a.row_runs || a.split != 1)) xl = 0;
  const int cx = xl && a.max_seg <= window(a.split) ? xl : 0;
  // dma -1 (default): register-staged x loaders; the split geometry's two
  // loader waves always stage by LDS-DMA (dispatch)
  const int dma = a.dma < 0 ? 0 : a.dma;
  const int ld = dma ? 1 : cx == 2 ? 2 : 0;
  (void)ld;
#ifndef HIPSPMV_EXPERIMENTAL_KERNELS
  // the product build instantiates what AUTO runs: the ordered geometry with its
  // register-staged loaders (CX 0; the ordered forms of the continuation options are experimental), the
  // split geometry with LDS-DMA loaders and the continuation its layout allows (5, else 3, else 0)
  if (a.split == 1 && !dma) {
    launch_one<T, 1, 0, 0>(a, s);
    return hipGetLastError();
  }
  if (a.split == 3 && a.map == 0 && (cx == 0 || cx == 3 || cx == 5)) {
    if (cx == 5)
      launch_one<T, 3, 1, 5>(a, s);
    else if (cx == 3)
      launch_one<T, 3, 1, 3>(a, s);
    else
      launch_one<T, 3, 1, 0>(a, s);
    return hipGetLastError();
  }
  return hipErrorNotSupported;
#else
  if (a.split == 1)
    dispatch<T, 1>(a, s, ld, cx);
  else if (a.split == 3 && a.map == 2 && cx == 5)  // (option "vcache_map" 2)
    launch_one<T, 3, 1, 5, 2>(a, s);
  else if (a.split == 3)
    dispatch<T, 3>(a, s, ld, cx);
  else if (cx == 5 && a.map == 1)  // four parts (probe, HIPSPMV_SPLIT4_VCACHE=1): LDS-DMA loaders, xlane 5
    launch_one<T, 4, 1, 5, 1>(a, s);
  else if (cx == 5)
    launch_one<T, 4, 1, 5, 0>(a, s);
  else  // four parts otherwise: k_vquad (csrc/vquad.hip) runs that layout
    return hipErrorInvalidValue;
  return hipGetLastError();
#endif
}

hipError_t launch_vcache(int dtype, const VcacheArgs& a, hipStream_t s) {
  return dtype ? launch_vcache<uint64_t>(a, s) : launch_vcache<double>(a, s);
}

template <typename T>
static hipError_t launch_vcache_profiled_t(const VcacheArgs& a, hipStream_t s) {
  const VcGeom g = a.split == 1 ? kVcOrdered : kVcSplit;
  if ((a.split != 1 && a.split != 3) || (a.split == 1 ? !a.partial : !a.tickets) ||
      !vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.panel,
                      a.split, g))
    return hipErrorInvalidValue;
  constexpr int P = 128;  // AB: profile stamps only
  const dim3 grid(a.nblocks * a.split), block(kVcThreads);
  if (a.split == 1) {
    hipLaunchKernelGGL((k_vcache<T, 1, VcCfg<1>::WL, VcCfg<1>::DE, VcCfg<1>::EPT, P>), grid, block, 0, s, a.seg,
                       a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial,
                       a.tickets, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad,
                       a.last, a.beta, a.nt_from, a.xmask);
  } else if (a.max_seg <= (uint32_t)((kVcThreads / 64 - VcCfg<3>::WL) * 64 * VcCfg<3>::EPT)) {
    hipLaunchKernelGGL((k_vcache<T, 3, VcCfg<3>::WL, VcCfg<3>::DE, VcCfg<3>::EPT, P, 0, false, 1, 3>), grid, block, 0,
                       s, a.seg, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out,
                       (T*)a.partial, a.tickets, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels,
                       a.part_panels, a.npad, a.last, a.beta, a.nt_from, a.xmask);
  } else {
    hipLaunchKernelGGL((k_vcache<T, 3, VcCfg<3>::WL, VcCfg<3>::DE, VcCfg<3>::EPT, P, 0, false, 1, 0>), grid, block, 0,
                       s, a.seg, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out,
                       (T*)a.partial, a.tickets, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels,
                       a.part_panels, a.npad, a.last, a.beta, a.nt_from, a.xmask);
  }
  return hipGetLastError();
}

hipError_t launch_vcache_profiled(int dtype, const VcacheArgs& a, hipStream_t s) {
  return dtype ? launch_vcache_profiled_t<uint64_t>(a, s) : launch_vcache_profiled_t<double>(a, s);
}

}  // namespace hipspmv
