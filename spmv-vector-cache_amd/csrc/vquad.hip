// k_vquad: the four-part LDS vector cache (HIPSPMV_KERNEL_VCACHE_SPLIT4,
// DESIGN.md §6.12) -- the round-4 FAST kernel for C3-like matrices.
//
// Why four parts.  A work unit keeps the y accumulators of R rows in LDS and
// streams its column part of x through LDS, so every CU moves 8 * cols / S
// bytes of x per launch besides its share of the entries.  Round 4's overlap
// probe (tools/overlap_probe.hip, profiles/r04) measured that the two streams
// do not overlap inside a CU -- their times add -- so the x bytes per CU are
// the lever: R = 16384 rows (128 KiB of y, the most LDS holds beside an x
// ring), S = 4 parts, 64 blocks x 4 = 256 units: 2 MiB of x per CU against
// 2.7 MiB for three parts of 12352 rows (free-running skeletons: 83 against
// 94 us).  What kept the round-2 four-part kernel slow (137 us) was its
// x ring: 1984-column panels with one panel in flight, waited for at every
// step.  Here the loader waves keep DX panels in flight in registers (asm
// loads, exact vmcnt waits) and only the store into LDS happens per step, so
// an x panel has DX steps to arrive.
//
// Work unit (b, h): rows [b*R, b*R + R), panels [vc_part_first(h), ...) of the
// kVcQuad layout (csrc/plan.cpp build_vcache per (block, panel) segment,
// re-placed by build_vcache_lanes: compute lane ct holds segment positions ct
// and CT + ct; code = col_local | row_local << 12 | LMORE | CONT | MORE).  The
// parts of a block run in dispatch slots i, i+8, i+16, i+24 (one XCD under
// round-robin placement: the combine's hand-off stays in one L2; speed only).
//
// Roles: waves [0, WL) stage x panels (LDS slot s & 1 holds panel s); waves
// [WL, 16) stream the unit's entries DE steps ahead (asm loads, exact waits)
// and apply them: every valid lane forms its rounded products from the LDS
// panel, a lane whose pair is one row (LMORE) adds it in registers, a rare
// longer run head (MORE) adds its run's next lanes by __shfl_down (the layout
// keeps such runs inside a wave), and owners update their y rows in LDS.  No
// two lanes own one row in a step, and the step barrier orders the steps.
// One s_barrier per panel.
//
// Combine (fixed order y = p0 + p1 + p2 + p3, deterministic): unit h owns
// quarter h of the block's rows and combines it; the other quarters it
// publishes (csrc/combine.h: bounded owner wait, publish-and-count fallback,
// so no deadlock rests on co-residency).
#include <hip/hip_runtime.h>

#include "combine.h"
#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"
#include "vc_map.h"

namespace hipspmv {

#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
namespace {

constexpr int VR = kVcQuad.rows, VP = kVcQuad.panel, SPLIT = 4;

// an asm-load ring value may be read (or its register reused) only after the
// wait that retired its load: the wait is followed by an empty asm that takes
// the value in and out, so no use moves above the wait and the register stays
// owned by the value until then (tools/vmcnt_check.py checks the build)
template <typename R>
__device__ __forceinline__ void tie(R& r) {
  asm volatile("" : "+v"(r));
}
__device__ __forceinline__ void tie(u64x2& r) {
  asm volatile("" : "+v"(r));
}
// entry loads through a buffer descriptor of the unit's entries: a lane past
// its step's segment gets an out-of-range offset and the load returns 0
// without a memory request, while every lane still issues the instruction
// (the ring's vmcnt counts stay exact).  Clamped loads instead re-read the
// next segment's entries: 1.68x the entry requests at four parts
// (the round-4 skeletons: entries alone 80 us barrier-stepped vs 59 us
// for a plain stream).
typedef unsigned int u32x4d __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4d buf_desc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  return u32x4d{(uint32_t)a, (uint32_t)(a >> 32), bytes, 0x00020000u};
}
__device__ __forceinline__ uint32_t bld_u32_nt(u32x4d d, uint32_t off) {
  uint32_t r;
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen nt" : "=v"(r) : "v"(off), "s"(d) : "memory");
  return r;
}
template <typename T>
__device__ __forceinline__ T bld_64_nt(u32x4d d, uint32_t off) {
  uint64_t r;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen nt" : "=v"(r) : "v"(off), "s"(d) : "memory");
  return __builtin_bit_cast(T, r);
}
// the same loads with the default policy: the lines allocate in the Infinity
// Cache and stay there across launches
__device__ __forceinline__ uint32_t bld_u32(u32x4d d, uint32_t off) {
  uint32_t r;
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(r) : "v"(off), "s"(d) : "memory");
  return r;
}
template <typename T>
__device__ __forceinline__ T bld_64(u32x4d d, uint32_t off) {
  uint64_t r;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(r) : "v"(off), "s"(d) : "memory");
  return __builtin_bit_cast(T, r);
}

constexpr uint32_t gcd_u(uint32_t a, uint32_t b) { return b ? gcd_u(b, a % b) : a; }
constexpr uint32_t lcm_u(uint32_t a, uint32_t b) { return a / gcd_u(a, b) * b; }

}  // namespace

// AB: ablation mask (timing probes only; results wrong unless 0): 1 no apply,
// 2 no x stores into LDS, 4 no combine (each part writes its own rows), 8 no
// step barrier, 16 x loads by LDS-DMA into the slots (timing only: DX > 1
// panels in flight overwrite each other), 32 no x loads, 64 no entry loads;
// 128 (results exact: the test of the combine's fallback) owners never wait.
// MAP 1: XCD-aware placement (csrc/vc_map.h: part h on XCDs 2h, 2h+1, so each
// XCD's L2 serves one quarter of x).  NTR: row blocks b < nt_from load their
// entries with the default policy (Infinity-Cache resident across launches),
// the others non-temporally (NTR 0: all non-temporal).  YADD: an owner adds
// its products to its y row with one LDS atomic (ds_add_f64 / ds_add_u64)
// instead of a read and a write -- the same one update per row and step, so
// the result is still deterministic.
template <typename T, int WL, int DX, int DE, int EPT, int AB = 0, int MAP = 0, bool NTR = false, bool YADD = false>
__global__ __launch_bounds__(kVcThreads) void k_vquad(const uint32_t* __restrict__ seg,
                                                       const uint32_t* __restrict__ ecode,
                                                       const T* __restrict__ evals, const T* __restrict__ x,
                                                       const T* __restrict__ y_in, T* __restrict__ y_out,
                                                       T* __restrict__ partial, uint32_t* __restrict__ tickets,
                                                       uint32_t* __restrict__ status, uint32_t rows, uint32_t cols,
                                                       uint32_t rows_per_block, uint32_t nblocks, uint32_t npanels,
                                                       uint32_t npad, uint32_t last, int beta, uint32_t nt_from) {
#pragma clang fp contract(off)
  constexpr int VT = kVcThreads, NW = VT / 64, WC = NW - WL;
  constexpr int LT = WL * 64, CT = WC * 64;
  constexpr uint32_t PAIRS = VP / 2;         // 16-byte pairs per panel
  constexpr int NJ = (PAIRS + LT - 1) / LT;  // pairs per loader lane per panel
  static_assert(VR * 8 + 2 * VP * 8 + kVcSegMax * 4 <= 163840, "LDS budget");
  static_assert(WL > 0 && WC > 0 && DX >= 2 && DE >= 2, "roles and rings");
  static_assert((DX - 1) * NJ < 64 && (DE - 1) * 2 * EPT < 64, "vmcnt field");
  __shared__ alignas(16) T ylds[VR];
  __shared__ alignas(16) T xb[2][VP];
  __shared__ uint32_t segl[kVcSegMax];

  const int t = threadIdx.x;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool loader = wv < (uint32_t)WL;  // wave-uniform role
  // unit i -> (b, h): the parts of a block are 8 dispatch slots apart
  uint32_t h, b;
  if (MAP == 1 && vc_map1_applies<SPLIT>(nblocks)) {
    vc_unit_map1<SPLIT>(blockIdx.x, b, h);
  } else {
    const uint32_t g8 = blockIdx.x / (8 * SPLIT), rem = blockIdx.x % (8 * SPLIT);
    const uint32_t nbg = min(8u, nblocks - g8 * 8);
    h = rem / nbg;
    b = g8 * 8 + rem % nbg;
  }
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry (workgroup-uniform, before any barrier)
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t p0 = vc_part_first(h, npanels, SPLIT);            // first global panel of this unit
  const uint32_t npu = vc_part_first(h + 1, npanels, SPLIT) - p0;  // >= 1 (vcache_grid_ok)
  const uint32_t* sp = seg + ((size_t)b * SPLIT + h) * (npad + 1);
  if ((uint32_t)t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = (beta && h == 0) ? y_in[r0 + i] : T(0);
  __syncthreads();  // segl visible; then each role's prologue, one barrier, the steps

  // every role runs the same padded step count (one barrier per step, no
  // early exit inside an unrolled group: the ring waits stay exact); in
  // barrier terms step s of both roles lies between the same two barriers
  constexpr uint32_t PER = lcm_u(DX, DE);
  const uint32_t nsteps = (npu + PER - 1) / PER * PER;

  auto barrier = [] {
    if (AB & 8) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };

  if (loader) {
    // ---- x panels: NJ 16-byte pairs per lane per panel, clamped in bounds
    // (branch-free), DX panels in flight in registers; in step s the panel
    // s + 1 is stored into slot (s + 1) & 1 (read last in step s - 1, closed
    // by that step's barrier) and panel s + 1 + DX is issued into its registers
    const uint32_t cmax = (cols - 2) & ~1u;
    const T xlast = __builtin_bit_cast(T, sld_64(x + cols - 1));  // scalar: no vmcnt slot in the ring
    u64x2 R[DX][NJ];
    auto issue = [&](uint32_t s, u64x2* r) {
      if (AB & 32) return;
      const uint32_t base = (p0 + min(s, npu - 1)) * VP;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const T* src = x + min(base + 2 * (t + j * LT), cmax);
        if (AB & 16) {
          const uint32_t c0 = (uint32_t)(j * LT) + wv * 64;  // this wave's 64 pairs of instruction j
          __builtin_amdgcn_global_load_lds((const void*)src,
                                           (__attribute__((address_space(3))) void*)(xb[s & 1] + 2 * min(c0, PAIRS - 64)),
                                           16, 0, 0);
        } else {
          asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[j]) : "v"(src) : "memory");
        }
      }
    };
    auto store = [&](uint32_t s, u64x2* r) {  // panel s into slot s & 1
      T* dst = xb[s & 1];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if ((j + 1) * LT <= (int)PAIRS || (uint32_t)(t + j * LT) < PAIRS)
          *reinterpret_cast<u64x2*>(&dst[2 * (t + j * LT)]) = r[j];
      if ((cols & 1) && p0 + s == npanels - 1) {  // odd cols: the last element from a scalar load
        const uint32_t sl = cols - 1 - (p0 + s) * VP;
        if ((uint32_t)t == (sl >> 1) % LT) dst[sl] = xlast;
      }
    };
    auto wait_slot = [&](u64x2* r) {  // the oldest panel of the ring landed, (DX - 1) * NJ loads younger
      if (AB & 32) return;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DX - 1) * NJ) : "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) tie(r[j]);
    };
#pragma unroll
    for (int d = 0; d < DX; ++d) issue(d, R[d]);
    wait_slot(R[0]);
    store(0, R[0]);
    issue(DX, R[0]);
    barrier();
    for (uint32_t base = 0; base < nsteps; base += DX) {
#pragma unroll
      for (int i = 0; i < DX; ++i) {
        const uint32_t s = base + i;  // ring slot of panel s + 1: (s + 1) % DX == (i + 1) % DX
        u64x2* r = R[(i + 1) % DX];
        wait_slot(r);
        if (!(AB & 2) && s + 1 < npu) store(s + 1, r);
        issue(s + 1 + DX, r);
        barrier();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped loads past the last panel
#pragma unroll
    for (int d = 0; d < DX; ++d)
#pragma unroll
      for (int j = 0; j < NJ; ++j) tie(R[d][j]);
  } else {
    // ---- entries: EPT per lane per step at clamped indices, DE steps in flight
    const int ct = t - LT;
    uint32_t EC[DE][EPT];
    T EV[DE][EPT];
    // the unit's entries [segl[0], segl[npu]) through two descriptors
    const uint32_t e0 = __builtin_amdgcn_readfirstlane(segl[0]),
                   ne = __builtin_amdgcn_readfirstlane(segl[npu]) - e0;  // wave-uniform: SGPR descriptors
    const u32x4d dcode = buf_desc(ecode + e0, 4 * ne), dvals = buf_desc(evals + e0, 8 * ne);
    uint32_t SB[DE], SE[DE];  // each ring slot's segment bounds (unit-relative), read once from LDS
    auto entries = [&](auto ntc) {
    auto issue = [&](uint32_t s, uint32_t* c, T* v, uint32_t& sb, uint32_t& se) {
      const uint32_t beg = segl[min(s, npad)] - e0, end = segl[min(s + 1, npad)] - e0;
      sb = beg;
      se = end;
      if (AB & 64) return;
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const uint32_t q = beg + ct + j * CT;
        const bool in = q < end;
        if constexpr (decltype(ntc)::value) {
          c[j] = bld_u32_nt(dcode, in ? 4 * q : 0x80000000u);
          v[j] = bld_64_nt<T>(dvals, in ? 8 * q : 0x80000000u);
        } else {
          c[j] = bld_u32(dcode, in ? 4 * q : 0x80000000u);
          v[j] = bld_64<T>(dvals, in ? 8 * q : 0x80000000u);
        }
      }
    };
    // step s over the build_vcache_lanes placement (lane ct holds positions ct
    // and CT + ct of the segment [beg, end)): both products from LDS panel
    // s & 1; a lane whose first entry carries kVqLMore adds its second entry
    // (the same row); a run head with kVcMore (runs longer than two, rare)
    // sums the next lanes of its wave by shuffles; every owner updates its y
    // row once.  No two owners share a row in a step.
    static_assert(EPT == 2, "build_vcache_lanes places two entries per lane");
    auto apply = [&](uint32_t s, uint32_t beg, uint32_t end, const uint32_t* c, const T* v) {
      const T* xs = xb[s & 1];
      T p[2], acc[2];
      bool own[2];
      uint32_t row[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t q = beg + ct + j * CT;
        const bool valid = q < end;
        p[j] = valid ? v[j] * xs[c[j] & 0xFFF] : T(0);  // rounded product (contract off)
        own[j] = valid && !(c[j] & kVcCont);
        row[j] = (c[j] >> 12) & 0x3FFF;
        acc[j] = own[j] ? (YADD ? p[j] : ylds[row[j]] + p[j]) : T(0);
      }
      if (own[0] && (c[0] & kVqLMore)) acc[0] = acc[0] + p[1];  // the lane's pair
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bool more = own[j] && (c[j] & kVcMore);
        for (uint32_t k = 1; __builtin_amdgcn_ballot_w64(more) != 0; ++k) {  // wave-uniform trip count
          const T pk = __shfl_down(p[j], k);
          const uint32_t ck = __shfl_down(c[j], k);
          if (more) {  // the layout keeps such a run inside its wave
            acc[j] = acc[j] + pk;
            more = (ck & kVcMore) != 0;
          }
        }
        if (own[j]) {
          if (YADD)
            __hip_atomic_fetch_add(&ylds[row[j]], acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            ylds[row[j]] = acc[j];
        }
      }
    };
#pragma unroll
    for (int d = 0; d < DE; ++d) issue(d, EC[d], EV[d], SB[d], SE[d]);
    barrier();
    for (uint32_t base = 0; base < nsteps; base += DE) {
#pragma unroll
      for (int i = 0; i < DE; ++i) {
        const uint32_t s = base + i;
        if (!(AB & 64)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DE - 1) * 2 * EPT) : "memory");  // step s landed
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
          tie(EC[i][j]);
          tie(EV[i][j]);
        }
        // apply before the slot's reload: the old values die first, so the
        // reload reuses their registers and the loop carries no copy of a
        // register whose load is in flight (vmcnt_check: a copy there reads it)
        if (!(AB & 1) && s < npu) apply(s, SB[i], SE[i], EC[i], EV[i]);
        issue(s + DE, EC[i], EV[i], SB[i], SE[i]);
        barrier();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int d = 0; d < DE; ++d)
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        tie(EC[d][j]);
        tie(EV[d][j]);
      }
    };
    if (!NTR || b >= nt_from)
      entries(std::true_type{});
    else
      entries(std::false_type{});
  }
  if (AB & 4) {
    __syncthreads();
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
    return;
  }
  // ---- combine: unit h owns quarter h of the block's rows (csrc/combine.h)
  __syncthreads();  // the entry waves' last (clamped) issue read segl after the final step barrier
  owner_combine<T, SPLIT, VT, (VR + 1) & ~1u, (AB & 128) != 0>(ylds, segl, partial, tickets + (size_t)SPLIT * b, b, h,
                                                               nblocks, nr, y_out + r0, t, status);
}

template <typename T, int WL, int DX, int DE, int AB = 0, int MAP = 0, bool NTR = false, bool YADD = false>
static void launch_cfg(const VcacheArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((k_vquad<T, WL, DX, DE, 2, AB, MAP, NTR, YADD>), dim3(a.nblocks * SPLIT), dim3(kVcThreads), 0, s,
                     a.seg, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial,
                     a.tickets, a.status, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.npad, a.last,
                     a.beta, a.nt_from);
}

// the register window (entries one step holds) of configuration v
static uint32_t vquad_window(int) { return kVqLanes * 2; }  // two slots per compute lane

template <typename T>
static hipError_t launch_vquad_t(const VcacheArgs& a, hipStream_t s) {
  if (!vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.panel,
                      a.split, kVcQuad) ||
      !a.status || a.max_seg > vquad_window(a.variant))
    return hipErrorInvalidValue;
  switch (a.variant) {  // (x panels in flight, entry steps in flight); 3 loader waves (the layout's CT)
    case 1: launch_cfg<T, 3, 4, 6>(a, s); break;
    case 2: launch_cfg<T, 3, 2, 6>(a, s); break;
    case 3: launch_cfg<T, 3, 3, 4>(a, s); break;
    case 4: launch_cfg<T, 3, 3, 8>(a, s); break;
    case 5: launch_cfg<T, 3, 4, 4>(a, s); break;
    case 17: launch_cfg<T, 3, 4, 3>(a, s); break;
    case 18: launch_cfg<T, 3, 2, 4>(a, s); break;
    case 19: launch_cfg<T, 3, 4, 5>(a, s); break;
    case 20: launch_cfg<T, 3, 3, 6, 128>(a, s); break;  // exact: every owner gives up waiting
    // round 5: XCD map (21), Infinity-Cache resident entries below nt_from (22, 23), LDS atomic y updates (24-26)
    case 21: launch_cfg<T, 3, 3, 6, 0, 1>(a, s); break;
    case 22: launch_cfg<T, 3, 3, 6, 0, 1, true>(a, s); break;
    case 23: launch_cfg<T, 3, 3, 6, 0, 0, true>(a, s); break;
    case 24: launch_cfg<T, 3, 3, 6, 0, 1, false, true>(a, s); break;
    case 25: launch_cfg<T, 3, 3, 6, 0, 1, true, true>(a, s); break;
    case 26: launch_cfg<T, 3, 3, 6, 0, 0, false, true>(a, s); break;
    // ablations (timing probes, wrong y): 6 no apply, 7 no x stores, 8 no combine,
    // 9 no apply and no x stores, 10 no step barriers (races), 11 skeleton (1|2|4),
    // 12 skeleton entries only, 13 skeleton x only, 14 skeleton x by LDS-DMA,
    // 15 skeleton without barriers, 16 ... and x by LDS-DMA
    case 6: launch_cfg<T, 3, 3, 6, 1>(a, s); break;
    case 7: launch_cfg<T, 3, 3, 6, 2>(a, s); break;
    case 8: launch_cfg<T, 3, 3, 6, 4>(a, s); break;
    case 9: launch_cfg<T, 3, 3, 6, 3>(a, s); break;
    case 10: launch_cfg<T, 3, 3, 6, 8>(a, s); break;
    case 11: launch_cfg<T, 3, 3, 6, 7>(a, s); break;
    case 12: launch_cfg<T, 3, 3, 6, 7 | 32>(a, s); break;
    case 13: launch_cfg<T, 3, 3, 6, 7 | 64>(a, s); break;
    case 14: launch_cfg<T, 3, 3, 6, 7 | 16>(a, s); break;
    case 15: launch_cfg<T, 3, 3, 6, 7 | 8>(a, s); break;
    case 16: launch_cfg<T, 3, 3, 6, 7 | 8 | 16>(a, s); break;
    default: launch_cfg<T, 3, 3, 6>(a, s); break;
  }
  return hipGetLastError();
}

uint32_t vquad_max_window(int variant) { return vquad_window(variant); }

hipError_t launch_vquad(int dtype, const VcacheArgs& a, hipStream_t s) {
  return dtype ? launch_vquad_t<uint64_t>(a, s) : launch_vquad_t<double>(a, s);
}
#else
// the product build: k_vquad is never chosen by AUTO -- built with make
// EXPERIMENTAL=1 only (lib/exp/libhipspmv.so); here selecting it reports "unsupported"
uint32_t vquad_max_window(int) { return 0; }
hipError_t launch_vquad(int, const VcacheArgs&, hipStream_t) { return hipErrorNotSupported; }
#endif

}  // namespace hipspmv
