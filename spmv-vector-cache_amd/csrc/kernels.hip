// HIPSpMV CSR kernels for gfx950 (MI355X, CDNA4, wave64).
//
// Each kernel computes y_out = (beta ? y_in : 0) + A*x over the CSR copy of A;
// the reference arithmetic is SoftwareSpMV::exec (software/SoftwareSpMV.cpp:
// 59-64): per row, products rounded then added in ascending column order.
// Compiled with -ffp-contract=off, and every body repeats
// `#pragma clang fp contract(off)`, so no a*b+c is fused.
//
//   k_csr_lane   ordered; one lane per CSR row, any matrix.      DESIGN.md §6.2
//   k_csr_vector fast; row groups, one wave each, wave-level segmented scan
//                with DPP row_shr / row_bcast.                   DESIGN.md §6.3
// The LDS vector-cache kernel is in vcache.hip.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"

namespace hipspmv {

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

// One wave's row group of y = A*x (plus y_in when beta).  KIND 0: plain
// csr_vector.  KIND 1: the wcsr segment pass -- entry
// (colind, vals) loads non-temporal, so the streamed entries do not push the
// current x window out of L2 (§6.10).  KIND 2: the wcsr reduce -- no values,
// each "entry" adds x[colind[e]] (a segment partial), so the same balanced
// groups and segmented scan sum every row's partials in a fixed order.
// out(r, v, nonempty): the result of row r of the group (v = its sum; a row
// with no entries passes nonempty false)
template <typename T, int KIND, typename XF, typename OUT>
__device__ __forceinline__ void csr_vector_rows(const uint32_t* __restrict__ rowptr,
                                                const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                XF xv, OUT out, uint32_t r0, uint32_t r1, uint32_t* heads) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const uint32_t base = rowptr[r0], n = rowptr[r1] - base;
  constexpr bool NTL = KIND == 1 || KIND == 3;  // entries non-temporal
  auto ci = [&](uint32_t e) { return NTL ? __builtin_nontemporal_load(colind + e) : colind[e]; };
  // the e-th term of the group's sums: a rounded product, or a partial
  auto term = [&](uint32_t e) -> T {
    if constexpr (KIND == 2) return xv(ci(e));
    else return (NTL ? __builtin_nontemporal_load(vals + e) : vals[e]) * xv(ci(e));
  };

  if (r1 - r0 == 1 && n > (uint32_t)kCvGroupNnz) {
    // long row: four interleaved lane accumulators, then a DPP wave reduction
    T a0 = T(0), a1 = T(0), a2 = T(0), a3 = T(0);
    uint32_t e = lane;
    for (; e + 192 < n; e += 256) {
      a0 = a0 + term(base + e);
      a1 = a1 + term(base + e + 64);
      a2 = a2 + term(base + e + 128);
      a3 = a3 + term(base + e + 192);
    }
    for (; e < n; e += 64) a0 = a0 + term(base + e);
    T s = (a0 + a1) + (a2 + a3);
    s = wave_segscan(s, lane == 0 ? 1u : 0u);  // one segment: lane 63 holds the total
    if (lane == 63) out(r0, s, true);
    return;
  }

  // multi-row group: <= 64 rows (lane i owns row r0+i), <= 256 nonzeros
  const bool own = (uint32_t)lane < r1 - r0;
  uint32_t rs = 0, re = 0;
  if (own) {
    rs = rowptr[r0 + lane] - base;
    re = rowptr[r0 + lane + 1] - base;
  }
  if (lane < kCvGroupNnz / 32) heads[lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (own && re > rs) atomicOr(&heads[rs >> 5], 1u << (rs & 31));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  T carry = T(0);
  if constexpr (KIND == 2 || KIND == 3) {
    // the wcsr reduce and k_wseg: every term of the group (<= 256) is loaded
    // before the scans, so a wave keeps four loads in flight instead of one
    // per round trip (k_wseg on C5 shard 0: 359.7 -> 322.4 us; the same in
    // the global segment pass, KIND 1, measured slower: 264.5 -> 270.8 us)
    constexpr int Q = kCvGroupNnz / 64;
    T pv[Q];
    if (n) {
#pragma unroll
      for (int q = 0; q < Q; ++q) pv[q] = term(base + min((uint32_t)(q * 64 + lane), n - 1));
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const uint32_t pb = (uint32_t)q * 64;
      if (pb >= n) break;
      const uint32_t e = pb + lane;
      T p = e < n ? pv[q] : T(0);
      const uint32_t f = e < n ? (heads[e >> 5] >> (e & 31)) & 1u : 0u;
      if (lane == 0 && !f) p = carry + p;
      p = wave_segscan(p, f);
      const uint32_t last = re - 1;
      const T tot = __shfl(p, (int)((last - pb) & 63));
      if (own && re > rs && last >= pb && last < pb + 64) out(r0 + lane, tot, true);
      carry = __shfl(p, 63);
    }
  } else {
    for (uint32_t pb = 0; pb < n; pb += 64) {
      const uint32_t e = pb + lane;
      T p = T(0);
      uint32_t f = 0;
      if (e < n) {
        p = term(base + e);
        f = (heads[e >> 5] >> (e & 31)) & 1u;
      }
      if (lane == 0 && !f) p = carry + p;
      p = wave_segscan(p, f);
      const uint32_t last = re - 1;  // this lane's row's final element (if its row is non-empty)
      const T tot = __shfl(p, (int)((last - pb) & 63));
      if (own && re > rs && last >= pb && last < pb + 64) out(r0 + lane, tot, true);
      carry = __shfl(p, 63);
    }
  }
  if (own && re == rs) out(r0 + lane, T(0), false);
}

// y[r] (+ y_in[r] when beta) for the row sums of a group
template <typename T>
struct RowOut {
  const T* y_in;
  T* y_out;
  int beta;
  __device__ void operator()(uint32_t r, T v, bool nonempty) const {
    y_out[r] = beta ? (nonempty ? y_in[r] + v : y_in[r]) : (nonempty ? v : T(0));
  }
};

// One wave's row group of y = A*x (plus y_in when beta).  KIND 0: plain
// csr_vector.  KIND 1: the wcsr segment pass -- entry
// (colind, vals) loads non-temporal, so the streamed entries do not push the
// current x window out of L2 (§6.10).  KIND 2: the wcsr reduce -- no values,
// each "entry" adds x[colind[e]] (a segment partial), so the same balanced
// groups and segmented scan sum every row's partials in a fixed order.
// (KIND 3, k_wseg: entries non-temporal, x from an LDS window.)
template <typename T, int KIND>
__device__ __forceinline__ void csr_vector_group(const uint32_t* __restrict__ rowptr,
                                                 const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                 const T* __restrict__ x, const T* __restrict__ y_in,
                                                 T* __restrict__ y_out, const uint32_t* __restrict__ groups,
                                                 uint32_t ngroups, int beta, uint32_t blk) {
  __shared__ uint32_t heads[4][kCvGroupNnz / 32];
  const int w = threadIdx.x >> 6;
  const uint32_t g = blk * 4 + w;
  if (g >= ngroups) return;  // wave-uniform; no workgroup barriers below
  csr_vector_rows<T, KIND>(rowptr, colind, vals, [&](uint32_t c) { return x[c]; }, RowOut<T>{y_in, y_out, beta},
                           groups[g], groups[g + 1], heads[w]);
}

// k_wseg (wcsr, LDS form): one chunk of one column window's segments per
// 1024-thread workgroup.  The window's 2^kWsLog2Window x values are staged in
// LDS once, then 16 waves run csr_vector groups over the chunk's segments
// with every gather served from LDS -- no L1/L2 request per gather.
template <typename T>
__global__ __launch_bounds__(1024) void k_wseg(const uint32_t* __restrict__ chunks,
                                               const uint32_t* __restrict__ groups,
                                               const uint32_t* __restrict__ rowptr,
                                               const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                               const T* __restrict__ x, uint32_t cols, T* __restrict__ ypart) {
  __shared__ T xw[1u << kWsLog2Window];
  __shared__ uint32_t heads[16][kCvGroupNnz / 32];
  const uint32_t* ck = chunks + 3 * (size_t)blockIdx.x;
  const uint32_t win = ck[0], g0 = ck[1], g1 = ck[2];
  const uint32_t c0 = win << kWsLog2Window, nc = min(1u << kWsLog2Window, cols - c0);
  for (uint32_t i = threadIdx.x; i < nc; i += 1024) xw[i] = x[c0 + i];
  __syncthreads();
  const int w = threadIdx.x >> 6;
  for (uint32_t g = g0 + (uint32_t)w; g < g1; g += 16)
    csr_vector_rows<T, 3>(rowptr, colind, vals, [&](uint32_t c) { return xw[c - c0]; },
                          RowOut<T>{(const T*)nullptr, ypart, 0}, groups[g], groups[g + 1], heads[w]);
}

// The wcsr segment pass's XCD placement (option "wcsr_xcd"):
// workgroup i runs on XCD i mod 8, so with xper = ceil(blocks / 8) it takes
// block (i mod 8) * xper + i / 8 -- XCD k walks the k-th contiguous eighth of
// the window-major groups, and its L2 gathers from those windows only instead
// of every XCD gathering from the window the whole chip is in.  The grid is
// 8 * xper; virtual blocks past the last return.  xper 0: block i.
__device__ __forceinline__ uint32_t wcsr_block(uint32_t xper) {
  return xper ? (blockIdx.x & 7u) * xper + (blockIdx.x >> 3) : blockIdx.x;
}

// k_wpass_hot (wcsr, hot-column form): one chunk (window,
// first group, end group) per 1024-thread workgroup, as k_wseg, but over the
// global-x windows: the window's HK hot columns (mark_hot_columns, csrc/plan.cpp)
// are gathered into LDS once, then 16 waves run the chunk's csr_vector groups
// with the hot entries' x from LDS and the others from global memory.  The
// same products in the same order as k_csr_vector over these groups.
// Measured slower than the product's segment pass on every C5 shard (§6.19):
// experimental build only (make EXPERIMENTAL=1, HIPSPMV_WCSR_HOT=K at create).
#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
template <typename T, uint32_t HK>
__global__ __launch_bounds__(1024) void k_wpass_hot(const uint32_t* __restrict__ chunks,
                                                    const uint32_t* __restrict__ groups,
                                                    const uint32_t* __restrict__ rowptr,
                                                    const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                    const T* __restrict__ x, const uint32_t* __restrict__ hot,
                                                    T* __restrict__ ypart) {
  __shared__ T xh[HK];
  __shared__ uint32_t heads[16][kCvGroupNnz / 32];
  const uint32_t* ck = chunks + 3 * (size_t)blockIdx.x;
  const uint32_t win = ck[0], g0 = ck[1], g1 = ck[2];
  const uint32_t* hw = hot + (size_t)win * HK;
  for (uint32_t i = threadIdx.x; i < HK; i += 1024) xh[i] = x[hw[i]];
  __syncthreads();
  const int w = threadIdx.x >> 6;
  auto xv = [&](uint32_t c) { return (c & kWcHotFlag) ? xh[c & (HK - 1)] : x[c]; };
  for (uint32_t g = g0 + (uint32_t)w; g < g1; g += 16)
    csr_vector_rows<T, 3>(rowptr, colind, vals, xv, RowOut<T>{(const T*)nullptr, ypart, 0}, groups[g], groups[g + 1],
                          heads[w]);
}
#endif

// NTE: the wcsr segment pass (KIND 1 above)
template <typename T, bool NTE = false>
__global__ __launch_bounds__(256) void k_csr_vector(const uint32_t* __restrict__ rowptr,
                                                     const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                     const T* __restrict__ x, const T* __restrict__ y_in,
                                                     T* __restrict__ y_out, const uint32_t* __restrict__ groups,
                                                     uint32_t ngroups, int beta) {
  csr_vector_group<T, NTE ? 1 : 0>(rowptr, colind, vals, x, y_in, y_out, groups, ngroups, beta, blockIdx.x);
}
// the wcsr segment pass with the XCD placement
template <typename T>
__global__ __launch_bounds__(256) void k_wpass_x(const uint32_t* __restrict__ rowptr,
                                                  const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                  const T* __restrict__ x, T* __restrict__ ypart,
                                                  const uint32_t* __restrict__ groups, uint32_t ngroups,
                                                  uint32_t xper) {
  csr_vector_group<T, 1>(rowptr, colind, vals, x, (const T*)nullptr, ypart, groups, ngroups, 0, wcsr_block(xper));
}

// k_wpass (wcsr segment pass with resident entries): the groups g <
// res_groups load their entries with the default cache policy, so those lines
// stay in the Infinity Cache across launches, the others non-temporally (the
// split vcache's residency); the arithmetic is k_csr_vector's
template <typename T>
__global__ __launch_bounds__(256) void k_wpass(const uint32_t* __restrict__ rowptr,
                                                const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                const T* __restrict__ x, T* __restrict__ ypart,
                                                const uint32_t* __restrict__ groups, uint32_t ngroups,
                                                uint32_t res_groups) {
  __shared__ uint32_t heads[4][kCvGroupNnz / 32];
  const int w = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x * 4 + w;
  if (g >= ngroups) return;  // wave-uniform
  auto xv = [&](uint32_t c) { return x[c]; };
  const RowOut<T> out{(const T*)nullptr, ypart, 0};
  if (g >= res_groups)
    csr_vector_rows<T, 1>(rowptr, colind, vals, xv, out, groups[g], groups[g + 1], heads[w]);
  else
    csr_vector_rows<T, 0>(rowptr, colind, vals, xv, out, groups[g], groups[g + 1], heads[w]);
}

// k_wpass_fill (wcsr segment pass, with the compact reduce): blocks below
// nfill write the rows without segments (y_in or +0.0, from the bitmap), the
// others run the segment pass's groups -- the streaming writes ride along
// the gather-bound pass instead of following the reduce (option wcsr_fill;
// the layout takes it when two thirds of the rows have no entry: C5 shard 7
// 270.3 -> 264.7 us, shards 5 / 6 (60 / 49 % empty) 2-3 us slower with it,
// fill blocks placed after the groups instead gained nothing;
// profiles/r05/logs/c5_ab_fill_*.log)
template <typename T>
__global__ __launch_bounds__(256) void k_wpass_fill(const uint32_t* __restrict__ rowptr,
                                                     const uint32_t* __restrict__ colind, const T* __restrict__ vals,
                                                     const T* __restrict__ x, T* __restrict__ ypart,
                                                     const uint32_t* __restrict__ groups, uint32_t ngroups,
                                                     const uint32_t* __restrict__ nebits, const T* __restrict__ y_in,
                                                     T* __restrict__ y_out, uint32_t rows, int beta, uint32_t nfill,
                                                     uint32_t xper) {
  const uint32_t v = wcsr_block(xper);  // (option wcsr_xcd: fill and group blocks placed by XCD eighths)
  if (v < nfill) {
    const uint32_t stride = nfill * 256;
    for (uint32_t r = v * 256 + threadIdx.x; r < rows; r += stride)
      if (!((nebits[r >> 5] >> (r & 31)) & 1u)) y_out[r] = beta ? y_in[r] : T(0);
    return;
  }
  __shared__ uint32_t heads[4][kCvGroupNnz / 32];
  const int w = threadIdx.x >> 6;
  const uint32_t g = (v - nfill) * 4 + w;
  if (g >= ngroups) return;  // wave-uniform
  csr_vector_rows<T, 1>(rowptr, colind, vals, [&](uint32_t c) { return x[c]; },
                        RowOut<T>{(const T*)nullptr, ypart, 0}, groups[g], groups[g + 1], heads[w]);
}

// k_wreduce (wcsr): y[r] = (y_in[r] +) the sum of row r's segment partials
// ypart[segidx[k]], k in [rowseg[r], rowseg[r+1]) (window order), over the
// reduce's own balanced row groups -- a fixed order, so wcsr is
// deterministic; a row with no segment gets y_in[r] (beta 1) or +0.0.
template <typename T>
__global__ __launch_bounds__(256) void k_wreduce(const uint32_t* __restrict__ rowseg,
                                                  const uint32_t* __restrict__ segidx, const T* __restrict__ ypart,
                                                  const T* __restrict__ y_in, T* __restrict__ y_out,
                                                  const uint32_t* __restrict__ groups, uint32_t ngroups, int beta) {
  csr_vector_group<T, 2>(rowseg, segidx, (const T*)nullptr, ypart, y_in, y_out, groups, ngroups, beta, blockIdx.x);
}

// k_wreduce_c (wcsr, compact reduce): the same sums as k_wreduce over groups
// of the rows that have segments only (rrow[i] the i-th such row, rsegc its
// segment offsets), so a group no longer spends lanes and a round trip per
// row on rows without entries -- C5's short-row shards are 50-70 % empty rows;
// blocks past red_blocks write the rows without segments (y_in or +0.0), one
// row per lane and grid-stride step, from the bitmap nebits.  The order of every row's sum is the
// group scan's, as in k_wreduce (deterministic; FAST bound).
template <typename T>
struct RowOutMapped {
  const uint32_t* rrow;
  const T* y_in;
  T* y_out;
  int beta;
  __device__ void operator()(uint32_t i, T v, bool nonempty) const {
    const uint32_t r = rrow[i];
    y_out[r] = beta ? (nonempty ? y_in[r] + v : y_in[r]) : (nonempty ? v : T(0));
  }
};
template <typename T>
__global__ __launch_bounds__(256) void k_wreduce_c(const uint32_t* __restrict__ rsegc,
                                                    const uint32_t* __restrict__ segidx, const T* __restrict__ ypart,
                                                    const uint32_t* __restrict__ rrow,
                                                    const uint32_t* __restrict__ nebits, const T* __restrict__ y_in,
                                                    T* __restrict__ y_out, const uint32_t* __restrict__ groups,
                                                    uint32_t ngroups, uint32_t red_blocks, uint32_t rows, int beta) {
  if (blockIdx.x < red_blocks) {
    __shared__ uint32_t heads[4][kCvGroupNnz / 32];
    const int w = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * 4 + w;
    if (g >= ngroups) return;  // wave-uniform; no workgroup barriers below
    csr_vector_rows<T, 2>(rsegc, segidx, (const T*)nullptr, [&](uint32_t c) { return ypart[c]; },
                          RowOutMapped<T>{rrow, y_in, y_out, beta}, groups[g], groups[g + 1], heads[w]);
    return;
  }
  const uint32_t stride = (gridDim.x - red_blocks) * 256;
  for (uint32_t r = (blockIdx.x - red_blocks) * 256 + threadIdx.x; r < rows; r += stride)
    if (!((nebits[r >> 5] >> (r & 31)) & 1u)) y_out[r] = beta ? y_in[r] : T(0);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
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

template <typename T>
hipError_t launch_wcsr(const WcsrArgs& a, hipStream_t s) {
  // the segment partials: csr_vector over A', beta 0, entries non-temporal;
  // the LDS form when the layout has window chunks
  if (a.nchunks && a.hot) {
#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
    if (a.hotk == kWcHotMax)
      hipLaunchKernelGGL((k_wpass_hot<T, kWcHotMax>), dim3(a.nchunks), dim3(1024), 0, s, a.chunks, a.groups,
                         a.seg_rowptr, a.seg_colind, (const T*)a.seg_vals, (const T*)a.x, a.hot, (T*)a.ypart);
    else
      hipLaunchKernelGGL((k_wpass_hot<T, 8192>), dim3(a.nchunks), dim3(1024), 0, s, a.chunks, a.groups,
                         a.seg_rowptr, a.seg_colind, (const T*)a.seg_vals, (const T*)a.x, a.hot, (T*)a.ypart);
#else
    return hipErrorNotSupported;  // (capi builds hot layouts only in the experimental build)
#endif
  } else if (a.nchunks)
    hipLaunchKernelGGL(k_wseg<T>, dim3(a.nchunks), dim3(1024), 0, s, a.chunks, a.groups, a.seg_rowptr, a.seg_colind,
                       (const T*)a.seg_vals, (const T*)a.x, a.cols, (T*)a.ypart);
  const bool fill_early = a.rrow && a.fill_early && !a.nchunks && !a.res_groups;
  const uint32_t nfill = std::min((a.rows + 255) / 256, 1024u);
  // option wcsr_xcd: the segment pass's blocks placed by XCD eighths (grid 8 * xper)
  auto xper_of = [&](uint32_t blocks) { return a.xcd ? (blocks + 7) / 8 : 0u; };
  auto grid_of = [&](uint32_t blocks) { return a.xcd ? 8 * xper_of(blocks) : blocks; };
  if (fill_early) {
    const uint32_t nb = nfill + (a.ngroups + 3) / 4;
    hipLaunchKernelGGL(k_wpass_fill<T>, dim3(grid_of(nb)), dim3(256), 0, s, a.seg_rowptr, a.seg_colind,
                       (const T*)a.seg_vals, (const T*)a.x, (T*)a.ypart, a.groups, a.ngroups, a.nebits,
                       (const T*)a.y_in, (T*)a.y_out, a.rows, a.beta, nfill, xper_of(nb));
  } else if (a.nchunks) {
    // (the chunked forms above wrote every segment partial; the hot form's colind carry the LDS flag and
    // must not reach a global-x pass)
  } else if (a.ngroups && a.xcd && !a.res_groups) {
    const uint32_t nb = (a.ngroups + 3) / 4;
    hipLaunchKernelGGL(k_wpass_x<T>, dim3(grid_of(nb)), dim3(256), 0, s, a.seg_rowptr, a.seg_colind,
                       (const T*)a.seg_vals, (const T*)a.x, (T*)a.ypart, a.groups, a.ngroups, xper_of(nb));
  } else if (a.ngroups && a.res_groups)
    hipLaunchKernelGGL(k_wpass<T>, dim3((a.ngroups + 3) / 4), dim3(256), 0, s, a.seg_rowptr, a.seg_colind,
                       (const T*)a.seg_vals, (const T*)a.x, (T*)a.ypart, a.groups, a.ngroups, a.res_groups);
  else if (a.ngroups)
    hipLaunchKernelGGL((k_csr_vector<T, true>), dim3((a.ngroups + 3) / 4), dim3(256), 0, s, a.seg_rowptr,
                       a.seg_colind, (const T*)a.seg_vals, (const T*)a.x, (const T*)nullptr, (T*)a.ypart,
                       a.groups, a.ngroups, 0);
  if (a.rrow) {
    // the fill: at most 1024 blocks, grid-stride (one block per 256 rows measured as a dispatch tail)
    const uint32_t red = (a.ncgroups + 3) / 4, fill = fill_early ? 0u : nfill;
    hipLaunchKernelGGL(k_wreduce_c<T>, dim3(red + fill), dim3(256), 0, s, a.rsegc, a.segidx, (const T*)a.ypart,
                       a.rrow, a.nebits, (const T*)a.y_in, (T*)a.y_out, a.cgroups, a.ncgroups, red, a.rows, a.beta);
  } else {
    hipLaunchKernelGGL(k_wreduce<T>, dim3((a.rgroups + 3) / 4), dim3(256), 0, s, a.rowseg, a.segidx,
                       (const T*)a.ypart, (const T*)a.y_in, (T*)a.y_out, a.reduce_groups, a.rgroups, a.beta);
  }
  return hipGetLastError();
}
hipError_t launch_wcsr(int dtype, const WcsrArgs& a, hipStream_t s) {
  return dtype ? launch_wcsr<uint64_t>(a, s) : launch_wcsr<double>(a, s);
}

hipError_t launch_csr_lane(int dtype, const CsrArgs& a, hipStream_t s) {
  return dtype ? launch_csr_lane<uint64_t>(a, s) : launch_csr_lane<double>(a, s);
}
hipError_t launch_csr_vector(int dtype, const CsrArgs& a, hipStream_t s) {
  return dtype ? launch_csr_vector<uint64_t>(a, s) : launch_csr_vector<double>(a, s);
}

}  // namespace hipspmv
