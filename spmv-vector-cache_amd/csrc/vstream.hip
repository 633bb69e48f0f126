// k_vstream: the LDS vector-cache SpMV with one role per wave.
//
// Same work units, layouts and arithmetic as k_vcache (csrc/vcache.hip): one
// 1024-thread workgroup owns a block of rows whose y accumulators live in LDS,
// x is streamed through two LDS panel slots, every gather of x and every y
// update is an LDS access, HBM sees each entry once.  What differs is the
// pipeline, rebuilt after the round-2 measurements (k_vcache's loader waves
// stream x at ~56 GB/s per CU against 100-135 GB/s for a plain stream, its
// compute waves drain their entry ring at the loop header):
//
//  * every wave streams both x and entries and applies entries -- no
//    producer/consumer split, so all 16 waves' loads are in flight at once and
//    no role idles at the barrier while the other works;
//  * both streams are register rings DX (x) and DE (entries) panels deep,
//    loaded branch-free at clamped addresses, with a step count padded to the
//    unroll, so no path leaves the unrolled group early (that early exit is
//    what made hipcc merge a vmcnt(0) into k_vcache's loop header) and the
//    compiler's own waits leave the younger panels in flight;
//  * a row run inside a segment (MORE) is finished by its wave in uniform
//    control flow from the products of the next lanes (v_readlane); a run
//    crossing into the next wave is finished with scalar loads (lgkmcnt), so
//    no vector load but the rings is ever waited for;
//  * one raw s_barrier per panel after an lgkmcnt(0): no fence that could ask
//    for vmcnt(0).
//
// SPLIT 1 (ordered geometry, 4096 rows): each row's products are added in
// ascending column order -- bit-identical to SoftwareSpMV.cpp:59-64.  SPLIT 2
// (8192 rows, two column halves): the deterministic p0 + p1 combine of
// k_vcache (FAST mode).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"
#include "vc_map.h"

namespace hipspmv {

template <int SPLIT>
struct VsCfg;
template <>
struct VsCfg<1> {
  static constexpr VcGeom G = kVcOrdered;
  static constexpr int DX = 2, DE = 4, EPT = 2;
};
template <>
struct VsCfg<2> {
  static constexpr VcGeom G = kVcSplit;
  static constexpr int DX = 4, DE = 4, EPT = 2;
};

// lane l's 64-bit value (readlane returns int: widen each half unsigned)
template <typename T>
__device__ __forceinline__ T readlane64(T v, uint32_t l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __builtin_bit_cast(T, (uint64_t)lo | ((uint64_t)hi << 32));
}

__device__ __forceinline__ void vs_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T, int SPLIT>
__global__ __launch_bounds__(kVcThreads) void k_vstream(const uint32_t* __restrict__ seg,
                                                         const uint32_t* __restrict__ ecode,
                                                         const T* __restrict__ evals, const T* __restrict__ x,
                                                         const T* __restrict__ y_in, T* __restrict__ y_out,
                                                         T* __restrict__ partial, uint32_t* __restrict__ tickets,
                                                         uint32_t rows, uint32_t cols, uint32_t rows_per_block,
                                                         uint32_t nblocks, uint32_t npanels, uint32_t part_panels,
                                                         uint32_t npad, uint32_t last, int beta) {
#pragma clang fp contract(off)
  constexpr int VR = VsCfg<SPLIT>::G.rows, VP = VsCfg<SPLIT>::G.panel;
  constexpr int DX = VsCfg<SPLIT>::DX, DE = VsCfg<SPLIT>::DE, EPT = VsCfg<SPLIT>::EPT;
  constexpr int VT = kVcThreads;
  constexpr uint32_t PAIRS = VP / 2;         // 16-byte x chunks per panel
  constexpr int NJ = (PAIRS + VT - 1) / VT;  // chunks per lane per panel
  constexpr int U = DX > DE ? DX : DE;       // unroll: every ring index static
  static_assert(U % DX == 0 && U % DE == 0, "ring depths divide the unroll");
  static_assert(VR * 8 + 2 * VP * 8 + kVcSegMax * 4 <= 163840, "LDS budget");
  __shared__ T ylds[VR];
  __shared__ T xb[2][VP];
  __shared__ uint32_t segl[kVcSegMax];

  const uint32_t t = threadIdx.x, lane = t & 63;
  uint32_t b, h;
  vc_unit_map0<SPLIT>(blockIdx.x, nblocks, b, h);  // the parts of a block are 8 dispatch slots apart
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry (workgroup-uniform, before any barrier)
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t p0 = h * part_panels;
  const uint32_t npu = min(part_panels, npanels - p0);  // >= 1 (vcache_eligible)
  const uint32_t* sp = seg + ((size_t)b * SPLIT + h) * (npad + 1);
  if (t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = (beta && h == 0) ? y_in[r0 + i] : T(0);

  // x panel p of this unit (clamped to its last panel), chunk t + j*VT
  const uint32_t cmax = (cols - 2) & ~1u;
  const T xlast = x[cols - 1];
  auto load_x = [&](uint32_t p, u64x2* r) {
    const uint32_t base = (p0 + min(p, npu - 1)) * VP;
#pragma unroll
    for (int j = 0; j < NJ; ++j) r[j] = *reinterpret_cast<const u64x2*>(x + min(base + 2 * (t + j * VT), cmax));
  };
  auto store_x = [&](uint32_t p, const u64x2* r) {
    T* dst = xb[p & 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if ((j + 1) * VT <= (int)PAIRS || t + j * VT < PAIRS) *reinterpret_cast<u64x2*>(&dst[2 * (t + j * VT)]) = r[j];
    if ((cols & 1) && p0 + p == npanels - 1) {  // odd cols: the last element from a scalar load
      const uint32_t slot = cols - 1 - (p0 + p) * VP;
      if (t == (slot >> 1) % VT) dst[slot] = xlast;
    }
  };
  // entries of step s at clamped indices (validity checked at use)
  auto load_e = [&](uint32_t s, uint32_t* c, T* v) {
    const uint32_t beg = segl[min(s, npad)];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t i = min(beg + t + j * VT, last);
      c[j] = ecode[i];
      v[j] = evals[i];
    }
  };
  auto apply = [&](uint32_t s, const uint32_t* c, const T* v) {
    const T* xs = xb[s & 1];
    const uint32_t beg = segl[s], end = segl[s + 1];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t q = beg + t + j * VT;
      const uint32_t code = c[j];
      const bool valid = q < end;
      const T p = valid ? v[j] * xs[code & 0xFFFF] : T(0);  // rounded product (contract off)
      const bool own = valid && !(code & kVcCont);
      const uint32_t row = (code >> 16) & 0x3FFF;
      T acc = own ? ylds[row] + p : T(0);
      // a run's continuation entries follow its head in entry order: finish each
      // run with the wave in uniform control flow -- the continuation products
      // read from the next lanes (v_readlane), past lane 63 from memory by
      // scalar loads (lgkmcnt: the vector rings stay in flight)
      for (uint64_t m = __builtin_amdgcn_ballot_w64(own && (code & kVcMore)); m; m &= m - 1) {  // rare
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        T a = readlane64(acc, l);
        uint32_t k = l + 1, cd;
        do {
          if (k < 64) {
            cd = (uint32_t)__builtin_amdgcn_readlane(code, k);
            a = a + readlane64(p, k);
          } else {
            const uint32_t i = (uint32_t)__builtin_amdgcn_readlane(q, l) + (k - l);
            cd = sld_32(ecode + i);
            a = a + __builtin_bit_cast(T, sld_64(evals + i)) * xs[cd & 0xFFFF];
          }
          ++k;
        } while (cd & kVcMore);
        if (lane == l) acc = a;
      }
      if (own) ylds[row] = acc;
    }
  };

  u64x2 RX[DX][NJ];  // RX[p % DX] holds x panel p from its load until it is stored
  uint32_t EC[DE][EPT];
  T EV[DE][EPT];  // EC/EV[s % DE] hold the entries of step s
#pragma unroll
  for (int d = 0; d < DX; ++d) load_x(d, RX[d]);
  __syncthreads();  // segl, ylds visible (no glds in flight: a plain barrier)
#pragma unroll
  for (int d = 0; d < DE; ++d) load_e(d, EC[d], EV[d]);
  store_x(0, RX[0]);
  load_x(DX, RX[0]);
  vs_barrier();
  const uint32_t nsteps = (npu + U - 1) / U * U;
  for (uint32_t base = 0; base < nsteps; base += U) {
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const uint32_t s = base + i;
      if (s < npu) apply(s, EC[i % DE], EV[i % DE]);
      load_e(s + DE, EC[i % DE], EV[i % DE]);
      if (s + 1 < npu) store_x(s + 1, RX[(i + 1) % DX]);  // slot (s+1)&1 was last read in step s-1
      load_x(s + 1 + DX, RX[(i + 1) % DX]);
      vs_barrier();
    }
  }
  if (SPLIT == 1) {
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
    return;
  }
  // ---- combine the two column halves, fixed order p0 + p1 (k_vcache's
  // validated hand-off: write-through partial stores, vmcnt drain, one ticket
  // add after the barrier, sc1 loads of the other partial by the second).
  uint64_t* mine = reinterpret_cast<uint64_t*>(partial) + (size_t)h * rows;
  for (uint32_t i = t; i < nr; i += VT)
    __hip_atomic_store(mine + r0 + i, __builtin_bit_cast(uint64_t, ylds[i]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    const uint32_t old = __hip_atomic_fetch_add(tickets + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (uint32_t)SPLIT - 1)
      __hip_atomic_store(tickets + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    segl[0] = old;
  }
  __syncthreads();
  if (segl[0] == 1) {
    const uint64_t* other = reinterpret_cast<const uint64_t*>(partial) + (size_t)(1 - h) * rows;
    for (uint32_t i = t; i < nr; i += VT) {
      const T o = __builtin_bit_cast(
          T, __hip_atomic_load(other + r0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const T m = ylds[i];
      y_out[r0 + i] = h == 0 ? m + o : o + m;
    }
  }
}

// Every segment must fit the register window: the kernel has no overflow path.
uint32_t vstream_window(int split) {
  return split == 1 ? (uint32_t)(kVcThreads * VsCfg<1>::EPT) : (uint32_t)(kVcThreads * VsCfg<2>::EPT);
}

template <typename T, int SPLIT>
static void launch_vs(const VcacheArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((k_vstream<T, SPLIT>), dim3(a.nblocks * SPLIT), dim3(kVcThreads), 0, s, a.seg, a.code,
                     (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, (T*)a.partial, a.tickets,
                     a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.last, a.beta);
}

hipError_t launch_vstream(int dtype, const VcacheArgs& a, hipStream_t s) {
  if (a.split != 1 && a.split != 2) return hipErrorInvalidValue;
  const VcGeom g = a.split == 1 ? kVcOrdered : kVcSplit;
  if (!vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.panel,
                      a.split, g))
    return hipErrorInvalidValue;
  if (a.max_seg > vstream_window(a.split)) return hipErrorInvalidValue;
  if (a.split == 1)
    dtype ? launch_vs<uint64_t, 1>(a, s) : launch_vs<double, 1>(a, s);
  else
    dtype ? launch_vs<uint64_t, 2>(a, s) : launch_vs<double, 2>(a, s);
  return hipGetLastError();
}

}  // namespace hipspmv
