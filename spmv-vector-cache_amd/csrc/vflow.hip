// k_vflow: the vector-cache SpMV with a flag-handed x ring.
//
// The LDS vector cache of k_vcache (csrc/vcache.hip; the reference's
// NoWMVectorCache.scala / SpMVFrontendNewCache.scala:102-151 idea: y kept on
// chip, x streamed) over four column parts of 16384-row blocks: each CU
// streams a quarter of x (x requests share each CU's L1->L2 slots with the
// entry stream), the parts combined in fixed order by the owner
// combine (csrc/combine.h).  What k_vcache's four-part forms lost to -- one
// workgroup barrier per step, with one x panel in flight --
// is replaced here:
//
//  * x panels of 1280 columns in a ring of kVfSlots LDS slots, filled by two
//    LDS-DMA loader waves up to two panels ahead.  A loader publishes a panel
//    by an LDS word per (slot, loader) once its DMA landed (vmcnt) and waits,
//    before refilling a slot, for an LDS count that the compute waves bump
//    when they are done reading it.  No s_barrier in the main loop.
//  * Compute wave w owns the block rows with vf_wave_of(row) == w: a y row is
//    read and written by one wave only, in step order, so the waves need not
//    keep step with each other (no lost update, no reordering: deterministic).
//    The layout (build_vflow) gives each (step, wave) its own group of at most
//    128 entries, two 64-lane slots loaded through buffer descriptors clamped
//    to the group (lanes past it issue no request), DE steps ahead.
//  * The apply is k_vcache's xlane-5 form: both slots' x and y reads together,
//    rounded products, a run head adds its first continuation from the next
//    lane by DPP (runs stay inside 16-lane rows) and longer runs by shuffles.
//
// Every flag wait is bounded (~20 ms; a normal one takes microseconds): a wait
// that gives up sets bit 1 of *status (stat "vflow_timeouts"; the results are
// then wrong, never a hang), and that wave waits for nothing after it.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "combine.h"
#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"
#include "vc_map.h"

namespace hipspmv {

#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
namespace {
constexpr int kVfVT = 1024;
constexpr uint32_t kVfSpinMax = 1u << 18;      // ~20 ms of s_sleep 1 polls: a wait past it is a fault
constexpr uint32_t kVfPairs = (uint32_t)kVfGeom.panel / 2;  // 16-byte chunks per panel
constexpr int kVfNdma = (int)(kVfPairs / 64);  // DMA wave-instructions per panel (one loader loads a panel)
static_assert(kVfPairs % 64 == 0, "a panel is whole DMA wave-instructions");
static_assert(kVfGeom.rows * 8 + kVfSlots * kVfGeom.panel * 8 + 64 <= 163840, "LDS budget");
static_assert(kVfLoaders + kVfWaves == kVfVT / 64, "wave roles");

__device__ __forceinline__ uint32_t vf_dpp_next32(uint32_t v) {  // lane l + 1 of its 16-lane row (15: 0)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, false);
}
template <typename T>
__device__ __forceinline__ T vf_dpp_next(T v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(T, (uint64_t)vf_dpp_next32((uint32_t)u) | (uint64_t)vf_dpp_next32((uint32_t)(u >> 32)) << 32);
}

// An LDS word store the compiler's waitcnt pass cannot see: issued right after the loader's counted
// vm_wait, it needs no more -- the pass would put vmcnt(0) before any LDS access that follows an
// LDS-DMA (it cannot tell the flag words from the panel slots), waiting for the next panel as well
__device__ __forceinline__ void vf_lds_store(uint32_t* p, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p;
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// waits until *p >= v (an LDS word other waves raise); false if it gave up.  The poll's read is asm for
// the same reason as vf_lds_store (in a loader it would otherwise wait for its panels in flight)
__device__ __forceinline__ bool vf_wait_ge(const uint32_t* p, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint32_t*)p;
  for (uint32_t spin = 0; spin < kVfSpinMax; ++spin) {
    uint32_t cur;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(cur) : "v"(a) : "memory");
    if (__builtin_amdgcn_readfirstlane(cur) >= v) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
}  // namespace

// DE: steps of entries in flight per compute wave (option "vflow_de").  PROF (option "vflow_prof",
// diagnostic): lane 0 of every wave adds s_memtime cycles to 4 counters at prof + 4 * (unit * 16 +
// wave): loader {waiting for a free slot, waiting for its DMA, total}, compute {waiting for a panel,
// applying, issuing its entry loads, total}
template <typename T, int MAP, int DE, bool PROF = false>
__global__ __launch_bounds__(kVfVT) void k_vflow(const uint32_t* __restrict__ wbeg, const uint32_t* __restrict__ wend,
                                                 const uint32_t* __restrict__ ecode, const T* __restrict__ evals,
                                                 const T* __restrict__ x, const T* __restrict__ y_in,
                                                 T* __restrict__ y_out, T* __restrict__ partial,
                                                 uint32_t* __restrict__ tickets, uint32_t* __restrict__ status,
                                                 uint32_t rows, uint32_t cols, uint32_t rows_per_block,
                                                 uint32_t nblocks, uint32_t npanels, uint32_t npad, int beta,
                                                 uint32_t nt_from, uint32_t* __restrict__ prof) {
#pragma clang fp contract(off)
  constexpr int VR = kVfGeom.rows, VP = kVfGeom.panel, S = kVfGeom.split, NS = kVfSlots;
  constexpr int WL = kVfLoaders, WC = kVfWaves;
  __shared__ alignas(16) T ylds[VR];
  __shared__ alignas(16) T xb[NS][VP];
  // [0, NS): full[slot] = 1 + the last panel published there; [8, 8 + NS): freed[slot] = compute-wave
  // releases of that slot so far; [8, 14): the combine's scratch once the main loop is over
  __shared__ uint32_t flags[16];
  uint32_t* const full = flags;
  uint32_t* const freed = flags + 8;
  uint32_t* const cscratch = flags + 8;  // reused by the combine once the main loop is over

  const int t = threadIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  uint32_t b, h;
  if (MAP == 1 && vc_map1_applies<S>(nblocks))
    vc_unit_map1<S>(blockIdx.x, b, h);  // XCDs 2h, 2h + 1 take part h: each XCD's L2 serves a quarter of x
  else
    vc_unit_map0<S>(blockIdx.x, nblocks, b, h);  // the parts of a block 8 dispatch slots apart
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry (workgroup-uniform, before any barrier)
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t p0 = vc_part_first(h, npanels, S);
  const uint32_t npu = vc_part_first(h + 1, npanels, S) - p0;  // >= 1 (vcache_grid_ok)
  for (uint32_t i = t; i < nr; i += kVfVT) ylds[i] = (beta && h == 0) ? y_in[r0 + i] : T(0);
  if (t < 16) flags[t] = 0;
  __syncthreads();
  uint64_t pc[4] = {0, 0, 0, 0};
  auto tnow = [] {
    asm volatile("" ::: "memory");
    const uint64_t v = __builtin_amdgcn_s_memtime();
    asm volatile("" ::: "memory");
    return v;
  };
  const uint64_t t_begin = PROF ? tnow() : 0;

  if (wave < (uint32_t)WL) {
    // ---- loader wave wl: the panels s = wl, wl + WL, ... of the part, each whole
    // into slot s % NS (64 16-byte pairs per wave-instruction, clamped in bounds;
    // odd cols: the last element patched after the DMA landed, by the lane owning
    // its pair), published as soon as it landed -- so WL panels are in flight
    // and no publish waits for a later panel's slot
    const uint32_t cmax = (cols - 2) & ~1u;
    const T xlast = x[cols - 1];
    auto dma = [&](uint32_t s) {
      const uint32_t base = (p0 + s) * VP;
      T* slot = xb[s % NS];
#pragma unroll
      for (int j = 0; j < kVfNdma; ++j) {
        const uint32_t c0 = j * 64;
        __builtin_amdgcn_global_load_lds((const void*)(x + min(base + 2 * (c0 + lane), cmax)),
                                         (__attribute__((address_space(3))) void*)(slot + 2 * c0), 16, 0, 0);
      }
    };
    auto publish = [&](uint32_t s) {  // panel s landed: patch, then its full word
      if ((cols & 1) && p0 + s == npanels - 1) {
        const uint32_t sl = cols - 1 - (p0 + s) * VP, c = sl >> 1;
        if ((c & 63) == lane) xb[s % NS][sl] = xlast;
      }
      // (no release fence: at workgroup scope it waits vmcnt(0) -- for the next panel's DMA too.  The
      // vm_wait before this retired the panel's LDS-DMA writes, and the asm's memory clobber keeps this
      // store after it)
      if (lane == 0) vf_lds_store(&full[s % NS], s + 1);
    };
    bool ok = true;
    for (uint32_t s = wave; s < npu; s += WL) {
      // the slot's previous panel (s - NS) released by every compute wave
      const uint64_t ta = PROF ? tnow() : 0;
      if (s >= (uint32_t)NS) ok = ok && vf_wait_ge(&freed[s % NS], (uint32_t)WC * (s / NS));
      const uint64_t tb = PROF ? tnow() : 0;
      dma(s);
      vm_wait<0>();  // (this wave's only loads in flight)
      publish(s);
      if (PROF) {
        const uint64_t tc = tnow();
        pc[0] += tb - ta;
        pc[1] += tc - tb;
      }
    }
    if (!ok && lane == 0) __hip_atomic_fetch_or(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    // ---- compute wave cw: its groups of the unit's steps, DE steps ahead
    const uint32_t cw = wave - WL, u = b * S + h;
    const uint32_t* gb = wbeg + ((size_t)u * WC + cw) * npad;
    const uint32_t* ge = wend + ((size_t)u * WC + cw) * npad;
    const uint32_t nsteps = (npu + DE - 1) / DE * DE;  // padded to the unroll: no early exit (exact waits)
    auto entries = [&](auto ntc) {
      constexpr int aux = decltype(ntc)::value ? 2 : 0;  // nt: kept out of the Infinity Cache
      uint32_t EC[DE][2], NB[DE];
      T EV[DE][2];
      // the group bounds of step s (scalar loads), one step before its entry loads need them
      auto bounds = [&](uint32_t s, uint32_t& e0, uint32_t& n) {
        const uint32_t k = min(s, npad - 1);
        e0 = gb[k];
        n = s < npu ? ge[k] - e0 : 0u;
      };
      auto load = [&](uint32_t e0, uint32_t n0, uint32_t* c, T* v, uint32_t& n) {
        n = n0;
        const __amdgpu_buffer_rsrc_t dc = buf_rsrc(ecode + e0, 4 * n), dv = buf_rsrc(evals + e0, 8 * n);
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // lanes past the group: out of the descriptor, no request
          c[j] = __builtin_amdgcn_raw_buffer_load_b32(dc, (int)(4 * (lane + 64 * j)), 0, aux);
          v[j] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(dv, (int)(8 * (lane + 64 * j)), 0, aux));
        }
      };
      auto apply = [&](uint32_t s, const uint32_t* c, const T* v, uint32_t n) {
        const T* xs = xb[s % NS];
        const int nj = n > 64 ? 2 : 1;  // wave-uniform: the second slot only when the group spills into it
        T xv[2], yv[2], p[2], acc[2];
        uint32_t row[2];
        bool own[2], more[2], edge[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= nj) break;
          row[j] = (c[j] >> 16) & 0x3FFF;
          xv[j] = xs[c[j] & 0xFFFF];  // a lane past the group holds code 0: reads x[0] / y[0], writes nothing
          yv[j] = ylds[row[j]];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= nj) break;
          const bool valid = lane + 64 * j < n;
          p[j] = valid ? v[j] * xv[j] : T(0);  // rounded product (contract off)
          own[j] = valid && !(c[j] & kVcCont);
          acc[j] = own[j] ? yv[j] + p[j] : T(0);
          more[j] = own[j] && (c[j] & kVcMore);
          const T p1 = vf_dpp_next(p[j]);
          const uint32_t c1 = vf_dpp_next32(c[j]);
          // lane 15 of a DPP row gets nothing from row_shl: a run that crosses into the next row (a
          // group the placement kept in (row, column) order) continues by shuffle from distance 1
          edge[j] = (lane & 15) == 15;
          if (more[j] && !edge[j]) {
            acc[j] = acc[j] + p1;
            more[j] = (c1 & kVcMore) != 0;
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= nj) break;
          for (uint32_t k = 1; __builtin_amdgcn_ballot_w64(more[j]) != 0; ++k) {  // runs of 3+, crossing runs
            const T pk = __shfl_down(p[j], k);
            const uint32_t ck = __shfl_down(c[j], k);
            if (more[j] && (k >= 2 || edge[j])) {
              acc[j] = acc[j] + pk;
              more[j] = (ck & kVcMore) != 0;
            }
          }
          if (own[j]) ylds[row[j]] = acc[j];
        }
      };
      bool ok = true;
      uint32_t be0, bn;
#pragma unroll
      for (int i = 0; i < DE; ++i) {
        bounds((uint32_t)i, be0, bn);
        load(be0, bn, EC[i], EV[i], NB[i]);
      }
      bounds((uint32_t)DE, be0, bn);
      for (uint32_t base = 0; base < nsteps; base += DE) {
#pragma unroll
        for (int i = 0; i < DE; ++i) {
          const uint32_t s = base + i;
          uint64_t ta = PROF ? tnow() : 0, tb = ta, tc = ta;
          if (s < npu) {
            ok = ok && vf_wait_ge(&full[s % NS], s + 1);  // after one wait gave up, none waits again
            if (PROF) tb = tnow();
            apply(s, EC[i], EV[i], NB[i]);
            // every x read of the slot retired, then release it to the loaders
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) __hip_atomic_fetch_add(&freed[s % NS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (PROF) tc = tnow();
          }
          load(be0, bn, EC[i], EV[i], NB[i]);  // step s + DE
          bounds(s + DE + 1, be0, bn);
          if (PROF) {
            const uint64_t td = tnow();
            pc[0] += tb - ta;
            pc[1] += tc - tb;
            pc[2] += td - tc;
          }
        }
      }
      if (!ok && lane == 0) __hip_atomic_fetch_or(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (b >= nt_from)
      entries(std::true_type{});
    else
      entries(std::false_type{});
  }
  if (PROF && lane == 0) {
    uint32_t* q = prof + 4 * ((size_t)(b * S + h) * 16 + wave);
    q[0] = (uint32_t)pc[0];
    q[1] = (uint32_t)pc[1];
    q[2] = (uint32_t)pc[2];
    q[3] = (uint32_t)(tnow() - t_begin);
  }
  __syncthreads();  // every y update in; the flag words are the combine's scratch from here
  owner_combine<T, S, kVfVT, (uint32_t)VR>(ylds, cscratch, partial, tickets + 4 * (size_t)b, b, h, nblocks, nr,
                                          y_out + r0, t);
}

template <typename T, int MAP, int DE>
static void launch_vflow_t(const VflowArgs& a, hipStream_t s) {
  if (a.prof)  // (diagnostic: the stamped instantiation)
    hipLaunchKernelGGL((k_vflow<T, MAP, DE, true>), dim3(a.nblocks * kVfGeom.split), dim3(kVfVT), 0, s, a.wbeg,
                       a.wend, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial,
                       a.tickets, a.status, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.npad, a.beta,
                       a.nt_from, a.prof);
  else
    hipLaunchKernelGGL((k_vflow<T, MAP, DE>), dim3(a.nblocks * kVfGeom.split), dim3(kVfVT), 0, s, a.wbeg, a.wend,
                       a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial,
                       a.tickets, a.status, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.npad, a.beta,
                       a.nt_from, (uint32_t*)nullptr);
}

hipError_t launch_vflow(int dtype, const VflowArgs& a, hipStream_t s) {
  if (!vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad,
                      (uint32_t)kVfGeom.panel, kVfGeom.split, kVfGeom) ||
      !a.status || a.cols < 2)
    return hipErrorInvalidValue;
  auto go = [&](auto t) {
    using T = decltype(t);
    switch (a.de * 2 + (a.map ? 1 : 0)) {
      case 4: launch_vflow_t<T, 0, 2>(a, s); break;
      case 5: launch_vflow_t<T, 1, 2>(a, s); break;
      case 6: launch_vflow_t<T, 0, 3>(a, s); break;
      case 7: launch_vflow_t<T, 1, 3>(a, s); break;
      case 9: launch_vflow_t<T, 1, 4>(a, s); break;
      case 16: launch_vflow_t<T, 0, 8>(a, s); break;
      case 17: launch_vflow_t<T, 1, 8>(a, s); break;
      default: launch_vflow_t<T, 0, 4>(a, s); break;
    }
  };
  if (dtype)
    go(uint64_t{});
  else
    go(double{});
  return hipGetLastError();
}

#else
// the product build: AUTO does not pick k_vflow -- built with make
// EXPERIMENTAL=1 only (lib/exp/libhipspmv.so); here selecting it reports "unsupported"
hipError_t launch_vflow(int, const VflowArgs&, hipStream_t) { return hipErrorNotSupported; }
#endif

}  // namespace hipspmv
