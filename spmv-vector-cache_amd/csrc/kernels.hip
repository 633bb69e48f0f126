// HIPSpMV device kernels for gfx950 (MI355X, CDNA4, wave64).
//
// Each kernel computes y_out = (beta ? y_in : 0) + A*x for its layout; the
// reference arithmetic is SoftwareSpMV::exec (software/SoftwareSpMV.cpp:59-64):
// per row, products rounded then added in ascending column order.  The file is
// compiled with -ffp-contract=off and every kernel body repeats
// `#pragma clang fp contract(off)`, so no a*b+c is fused (tests/ check the
// ordered kernels bit-for-bit against the oracle).
//
//   k_vcache     ordered; x panels and the row block's y accumulators staged in
//                LDS (the GPU analogue of the reference's vector cache,
//                chisel/cache-new/NoWMVectorCache.scala); one 1024-thread
//                workgroup per row block.                        DESIGN.md §3.1
//   k_csr_lane   ordered; one lane per CSR row, any matrix.      DESIGN.md §3.2
//   k_csr_vector fast; row groups, one wave each, wave-level segmented scan
//                with DPP row_shr / row_bcast.                   DESIGN.md §3.3
#include <hip/hip_runtime.h>

#include "hipspmv_internal.h"
#include "kernels.h"

namespace hipspmv {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T madd(T acc, T a, T b) {
#pragma clang fp contract(off)
  const T p = a * b;  // rounded (f64) / truncated mod 2^64 (u64) before the add
  return acc + p;
}

// ---------------------------------------------------------------------------
// k_vcache
// ---------------------------------------------------------------------------
// One workgroup per work unit (row block b, column part h).  Per panel of VP
// columns: x[panel] -> LDS (register-staged, kVcDepth panels ahead), the
// unit's entries of that panel (same prefetch distance, so the in-order
// vmcnt never makes a young load wait behind an old one) each add
// val * x_lds[col] into y_lds[row]; one barrier per panel.  SPLIT == 2: the
// two column parts of a block run in workgroups i and i+8 (one XCD under
// round-robin dispatch, speed only), each publishes its partial and the
// second to arrive writes y = p0 + p1 (agent-scope release/acquire ticket,
// MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility").
template <typename T, int VR, int VP, int SPLIT>
__global__ __launch_bounds__(kVcThreads) void k_vcache(const uint32_t* __restrict__ seg,
                                                        const uint32_t* __restrict__ ecode,
                                                        const T* __restrict__ evals, const T* __restrict__ x,
                                                        const T* __restrict__ y_in, T* __restrict__ y_out,
                                                        T* __restrict__ partial, uint32_t* __restrict__ tickets,
                                                        uint32_t rows, uint32_t cols, uint32_t rows_per_block,
                                                        uint32_t nblocks, uint32_t npanels, uint32_t part_panels,
                                                        uint32_t npad, uint32_t last, int beta) {
#pragma clang fp contract(off)
  constexpr int VT = kVcThreads, D = kVcDepth, EPT = kVcEpt;
  constexpr uint32_t PAIRS = VP / 2;  // 16-byte pairs per panel
  constexpr int NJ = (PAIRS + VT - 1) / VT;
  static_assert(VR * 8 + 2 * VP * 8 + kVcSegMax * 4 <= 163840, "LDS budget");
  __shared__ T ylds[VR];
  __shared__ T xb[2][VP];
  __shared__ uint32_t segl[kVcSegMax];

  const int t = threadIdx.x;
  uint32_t b = blockIdx.x, h = 0;
  if (SPLIT == 2) {  // unit i -> (b, h): parts of one block are 8 dispatch slots apart
    const uint32_t g = blockIdx.x / 16, rem = blockIdx.x % 16;
    const uint32_t nbg = min(8u, nblocks - g * 8);
    h = rem / nbg;
    b = g * 8 + rem % nbg;
  }
  const uint32_t r0 = b * rows_per_block;
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t p0 = h * part_panels;                   // first global panel of this unit
  const uint32_t npu = min(part_panels, npanels - p0);   // >= 1 (vcache_eligible)
  const uint32_t* sp = seg + ((size_t)b * SPLIT + h) * (npad + 1);
  if ((uint32_t)t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = (beta && h == 0) ? y_in[r0 + i] : T(0);

  // x panel staging: branch-free 16-byte loads clamped to the last in-bounds
  // pair (so no divergent path rewrites an in-flight load register); for odd
  // cols the final element is patched from a scalar load by the thread owning
  // its LDS slot.
  const uint32_t cmax = (cols - 2) & ~1u;
  const T xlast = x[cols - 1];
  auto load_x = [&](uint32_t s, u64x2* r) {
    const uint32_t base = (p0 + min(s, npu - 1)) * VP;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      r[j] = *reinterpret_cast<const u64x2*>(x + min(base + 2 * (t + j * VT), cmax));
  };
  auto store_x = [&](uint32_t s, const u64x2* r) {
    T* dst = xb[s & 1];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if ((j + 1) * VT <= (int)PAIRS || (uint32_t)(t + j * VT) < PAIRS)
        *reinterpret_cast<u64x2*>(&dst[2 * (t + j * VT)]) = r[j];
    if ((cols & 1) && p0 + s == npanels - 1) {
      const uint32_t slot = cols - 1 - (p0 + s) * VP;
      if ((uint32_t)t == (slot >> 1) % VT) dst[slot] = xlast;
    }
  };
  // entries: branch-free loads at clamped indices, validity checked at use
  auto load_e = [&](uint32_t s, uint32_t* c, T* v) {
    const uint32_t beg = segl[min(s, npad)];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t i = min(beg + t + j * VT, last);
      c[j] = __builtin_nontemporal_load(ecode + i);
      v[j] = __builtin_nontemporal_load(evals + i);
    }
  };
  // a row run: its first entry is held by this thread; continuation entries
  // (MORE) are read back from memory (rare: >1 entry of a row in one panel)
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

  u64x2 X[D][NJ];
  uint32_t EC[D][EPT];
  T EV[D][EPT];
  __syncthreads();  // segl visible
  load_x(0, X[0]);
  store_x(0, X[0]);
#pragma unroll
  for (int i = 0; i < D; ++i) {
    load_e(i, EC[i], EV[i]);
    load_x(i + 1, X[(i + 1) % D]);
  }
  __syncthreads();
  for (uint32_t base = 0; base < npad; base += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const uint32_t s = base + i;
      const T* xs = xb[s & 1];
      const uint32_t beg = segl[s], end = segl[s + 1];
#pragma unroll
      for (int j = 0; j < EPT; ++j) {
        const uint32_t q = beg + t + j * VT;
        if (q < end && !(EC[i][j] & kVcCont)) run(q, EC[i][j], EV[i][j], xs);
      }
      for (uint32_t q = beg + EPT * VT + t; q < end; q += VT) {  // overflow beyond the register window
        const uint32_t code = ecode[q];
        if (!(code & kVcCont)) run(q, code, evals[q], xs);
      }
      load_e(s + D, EC[i], EV[i]);
      if (s + 1 < npu) store_x(s + 1, X[(i + 1) % D]);
      load_x(s + 1 + D, X[(i + 1) % D]);
      __syncthreads();
    }
  }
  if (SPLIT == 1) {
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
    return;
  }
  // ---- combine the two column parts (fixed order p0 + p1) ----
  T* mine = partial + (size_t)h * rows;
  for (uint32_t i = t; i < nr; i += VT) mine[r0 + i] = ylds[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(tickets + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(tickets + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
    }
    segl[0] = old;
  }
  __syncthreads();
  if (segl[0] == 1) {
    const T* other = partial + (size_t)(1 - h) * rows;
    for (uint32_t i = t; i < nr; i += VT) {
      const T o = other[r0 + i], m = ylds[i];
      y_out[r0 + i] = h == 0 ? m + o : o + m;
    }
  }
}

// ---------------------------------------------------------------------------
// k_csr_lane: ordered, one lane per row
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_csr_lane(const uint32_t* __restrict__ rowptr,
                                                   const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                   const T* __restrict__ x, const T* __restrict__ y_in,
                                                   T* __restrict__ y_out, uint32_t rows, int beta) {
#pragma clang fp contract(off)
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  T acc = beta ? y_in[r] : T(0);
  const uint32_t e1 = rowptr[r + 1];
  for (uint32_t e = rowptr[r]; e < e1; ++e) acc = madd(acc, vals[e], x[colind[e]]);
  y_out[r] = acc;
}

// ---------------------------------------------------------------------------
// k_csr_vector: fast, wave per row group, DPP segmented scan
// ---------------------------------------------------------------------------
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  // lanes whose source is outside the row, or whose row is masked off, read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK, typename T>
__device__ __forceinline__ T dpp64(T v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)u);
  const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(u >> 32));
  return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
}
// one step of an inclusive segmented scan: (v,f) <- (v',f') (+) (v,f)
template <int CTRL, int ROW_MASK, typename T>
__device__ __forceinline__ void seg_step(T& v, uint32_t& f) {
#pragma clang fp contract(off)
  const T vp = dpp64<CTRL, ROW_MASK>(v);
  const uint32_t fp = dpp32<CTRL, ROW_MASK>(f);
  v = f ? v : vp + v;
  f |= fp;
}
// Inclusive segmented sum across the 64 lanes (segment heads have f = 1):
// row_shr:1,2,4,8 scan each 16-lane DPP row, then row_bcast:15 carries the
// row tails into rows 1 and 3 and row_bcast:31 carries lane 31 into rows 2
// and 3 (gfx9 DPP).
template <typename T>
__device__ __forceinline__ T wave_segscan(T v, uint32_t f) {
  seg_step<0x111, 0xF>(v, f);  // row_shr:1
  seg_step<0x112, 0xF>(v, f);  // row_shr:2
  seg_step<0x114, 0xF>(v, f);  // row_shr:4
  seg_step<0x118, 0xF>(v, f);  // row_shr:8
  seg_step<0x142, 0xA>(v, f);  // row_bcast:15 -> rows 1,3
  seg_step<0x143, 0xC>(v, f);  // row_bcast:31 -> rows 2,3
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void k_csr_vector(const uint32_t* __restrict__ rowptr,
                                                     const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                     const T* __restrict__ x, const T* __restrict__ y_in,
                                                     T* __restrict__ y_out, const uint32_t* __restrict__ groups,
                                                     uint32_t ngroups, int beta) {
#pragma clang fp contract(off)
  __shared__ uint32_t heads[4][kCvGroupNnz / 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x * 4 + w;
  if (g >= ngroups) return;  // wave-uniform; no workgroup barriers below
  const uint32_t r0 = groups[g], r1 = groups[g + 1];
  const uint32_t base = rowptr[r0], n = rowptr[r1] - base;

  if (r1 - r0 == 1 && n > (uint32_t)kCvGroupNnz) {
    // long row: four interleaved lane accumulators, then a DPP wave reduction
    T a0 = T(0), a1 = T(0), a2 = T(0), a3 = T(0);
    uint32_t e = lane;
    for (; e + 192 < n; e += 256) {
      a0 = madd(a0, vals[base + e], x[colind[base + e]]);
      a1 = madd(a1, vals[base + e + 64], x[colind[base + e + 64]]);
      a2 = madd(a2, vals[base + e + 128], x[colind[base + e + 128]]);
      a3 = madd(a3, vals[base + e + 192], x[colind[base + e + 192]]);
    }
    for (; e < n; e += 64) a0 = madd(a0, vals[base + e], x[colind[base + e]]);
    T s = (a0 + a1) + (a2 + a3);
    s = wave_segscan(s, lane == 0 ? 1u : 0u);  // one segment: lane 63 holds the total
    if (lane == 63) y_out[r0] = beta ? y_in[r0] + s : s;
    return;
  }

  // multi-row group: <= 64 rows (lane i owns row r0+i), <= 256 nonzeros
  const bool own = (uint32_t)lane < r1 - r0;
  uint32_t rs = 0, re = 0;
  if (own) {
    rs = rowptr[r0 + lane] - base;
    re = rowptr[r0 + lane + 1] - base;
  }
  if (lane < kCvGroupNnz / 32) heads[w][lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (own && re > rs) atomicOr(&heads[w][rs >> 5], 1u << (rs & 31));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  T carry = T(0);
  for (uint32_t pb = 0; pb < n; pb += 64) {
    const uint32_t e = pb + lane;
    T p = T(0);
    uint32_t f = 0;
    if (e < n) {
      p = vals[base + e] * x[colind[base + e]];
      f = (heads[w][e >> 5] >> (e & 31)) & 1u;
    }
    if (lane == 0 && !f) p = carry + p;
    p = wave_segscan(p, f);
    const uint32_t last = re - 1;  // this lane's row's final element (if its row is non-empty)
    const T tot = __shfl(p, (int)((last - pb) & 63));
    if (own && re > rs && last >= pb && last < pb + 64) y_out[r0 + lane] = beta ? y_in[r0 + lane] + tot : tot;
    carry = __shfl(p, 63);
  }
  if (own && re == rs) y_out[r0 + lane] = beta ? y_in[r0 + lane] : T(0);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <typename T>
hipError_t launch_vcache(const VcacheArgs& a, hipStream_t s) {
  const uint32_t units = a.nblocks * a.split;
  if (a.split == 1)
    hipLaunchKernelGGL((k_vcache<T, kVcOrdered.rows, kVcOrdered.panel, 1>), dim3(units), dim3(kVcThreads), 0, s,
                       a.seg, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out,
                       (T*)a.partial, a.tickets, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels,
                       a.part_panels, a.npad, a.last, a.beta);
  else
    hipLaunchKernelGGL((k_vcache<T, kVcSplit.rows, kVcSplit.panel, 2>), dim3(units), dim3(kVcThreads), 0, s,
                       a.seg, a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out,
                       (T*)a.partial, a.tickets, a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels,
                       a.part_panels, a.npad, a.last, a.beta);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_csr_lane(const CsrArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_csr_lane<T>, dim3((a.rows + 255) / 256), dim3(256), 0, s, a.rowptr, a.colind,
                     (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.rows, a.beta);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_csr_vector(const CsrArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_csr_vector<T>, dim3((a.ngroups + 3) / 4), dim3(256), 0, s, a.rowptr, a.colind,
                     (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.groups, a.ngroups, a.beta);
  return hipGetLastError();
}

hipError_t launch_vcache(int dtype, const VcacheArgs& a, hipStream_t s) {
  return dtype ? launch_vcache<uint64_t>(a, s) : launch_vcache<double>(a, s);
}
hipError_t launch_csr_lane(int dtype, const CsrArgs& a, hipStream_t s) {
  return dtype ? launch_csr_lane<uint64_t>(a, s) : launch_csr_lane<double>(a, s);
}
hipError_t launch_csr_vector(int dtype, const CsrArgs& a, hipStream_t s) {
  return dtype ? launch_csr_vector<uint64_t>(a, s) : launch_csr_vector<double>(a, s);
}

}  // namespace hipspmv
