// Matrix preprocessing scans on the GPU: the statistics SoftwareSpMV reports
// beside its SpMV time (software/SoftwareSpMV.cpp:72-95) and the cold-miss-skip
// marking the NewCache backends consume (software/SparseMatrix.cpp:52-90).
//
//   maxColSpan  (SparseMatrix.cpp:110-119): max over columns of
//               inds[colptr[c+1]-1] - inds[colptr[c]] (u32 arithmetic).
// Row ids are read with bits 30-31 masked throughout: the reference's values
// on an unmarked matrix, which is how SoftwareSpMV calls them.
//   maxAlive    (SparseMatrix.cpp:92-108): in storage order, a row is "alive"
//               from its first entry (bit 31) to its last (bit 30); the max
//               number alive after each entry.  Computed from per-row first and
//               last entry positions (atomicMin/Max), a +1/-1 delta stream and
//               an ordered (sum, max-prefix) reduction -- no global scan.
//   markRowStarts (SparseMatrix.cpp:52-90): OR 1<<shift into the first
//               (reverse: last) entry of every row.
//
// All three are HBM-bound integer streams (4 B per column / entry plus the
// per-row position arrays); they run once per matrix, off the SpMV path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "hipspmv.h"
#include "hipspmv_internal.h"

namespace hipspmv {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;  // entries per thread in the alive reduction
constexpr uint32_t kRowMask = 0x3FFFFFFFu;

// (sum, max-prefix) of a +1/-1 stream, the empty prefix included (so mp >= 0).
// combine(a, b) is associative, not commutative: a comes first.
struct SumMax {
  int64_t sum, mp;
};
__device__ inline SumMax combine(SumMax a, SumMax b) { return {a.sum + b.sum, max(a.mp, a.sum + b.mp)}; }

__device__ inline SumMax wave_combine_down(SumMax v) {
  // ordered reduction: after step s, lane i (i % 2s == 0) holds lanes [i, i+2s)
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    SumMax o{__shfl_down(v.sum, s), __shfl_down(v.mp, s)};
    if ((threadIdx.x & 63) + s < 64) v = combine(v, o);
  }
  return v;
}

__device__ inline SumMax block_combine(SumMax v) {
  __shared__ SumMax waves[kThreads / 64];
  v = wave_combine_down(v);
  if ((threadIdx.x & 63) == 0) waves[threadIdx.x >> 6] = v;
  __syncthreads();
  SumMax t{0, 0};
  if (threadIdx.x == 0)
    for (int w = 0; w < kThreads / 64; ++w) t = combine(t, waves[w]);
  return t;  // valid in thread 0
}

// MODE bit 0: record first positions, bit 1: record last positions.
template <int MODE>
__global__ void __launch_bounds__(kThreads) k_first_last(const uint32_t* __restrict__ inds, uint32_t nnz,
                                                         uint32_t rows, uint32_t* __restrict__ first,
                                                         uint32_t* __restrict__ last, uint32_t* __restrict__ bad) {
  for (uint64_t e = blockIdx.x * kThreads + threadIdx.x; e < nnz; e += gridDim.x * kThreads) {
    const uint32_t r = inds[e] & kRowMask;
    if (r >= rows) {
      atomicOr(bad, 1u);
      continue;
    }
    if (MODE & 1) atomicMin(first + r, (uint32_t)e);
    if (MODE & 2) atomicMax(last + r, (uint32_t)e);
  }
}

// delta[first[r]] = +1, delta[last[r]] = -1 (nothing for a one-entry row: its
// +1 and -1 land on the same entry before the max is taken).  Positions of
// different rows are distinct, so plain stores suffice.
__global__ void __launch_bounds__(kThreads) k_alive_delta(const uint32_t* __restrict__ first,
                                                          const uint32_t* __restrict__ last, uint32_t rows,
                                                          int8_t* __restrict__ delta) {
  for (uint32_t r = blockIdx.x * kThreads + threadIdx.x; r < rows; r += gridDim.x * kThreads) {
    const uint32_t f = first[r], l = last[r];
    if (f == 0xFFFFFFFFu || f == l) continue;  // row absent / single entry
    delta[f] = 1;
    delta[l] = -1;
  }
}

// Block b reduces entries [b*kThreads*kItems, ...) to one SumMax, in order.
__global__ void __launch_bounds__(kThreads) k_alive_blocks(const int8_t* __restrict__ delta, uint32_t nnz,
                                                           SumMax* __restrict__ out) {
  static_assert(kItems == 16, "one 16-byte load per thread");
  const uint64_t base = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) * kItems;
  union {
    uint4 q;
    int8_t b[kItems];
  } d;
  if (base + kItems <= nnz) {
    d.q = *reinterpret_cast<const uint4*>(delta + base);
  } else {
#pragma unroll
    for (int i = 0; i < kItems; ++i) d.b[i] = base + i < nnz ? delta[base + i] : 0;
  }
  SumMax v{0, 0};
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    v.sum += d.b[i];
    v.mp = max(v.mp, v.sum);
  }
  v = block_combine(v);
  if (threadIdx.x == 0) out[blockIdx.x] = v;
}

// One workgroup folds the per-block pairs in order: thread t owns a
// contiguous run of them.
__global__ void __launch_bounds__(kThreads) k_alive_final(const SumMax* __restrict__ parts, uint32_t n,
                                                          uint32_t* __restrict__ result) {
  const uint32_t per = (n + kThreads - 1) / kThreads;
  const uint32_t b0 = threadIdx.x * per, b1 = min(n, b0 + per);
  SumMax v{0, 0};
  for (uint32_t b = b0; b < b1; ++b) v = combine(v, parts[b]);
  v = block_combine(v);
  if (threadIdx.x == 0) *result = (uint32_t)v.mp;
}

__global__ void __launch_bounds__(kThreads) k_col_span(const uint32_t* __restrict__ colptr,
                                                       const uint32_t* __restrict__ inds, uint32_t cols,
                                                       uint32_t nnz, uint32_t* __restrict__ result) {
  uint32_t best = 0;
  for (uint32_t c = blockIdx.x * kThreads + threadIdx.x; c < cols; c += gridDim.x * kThreads) {
    const uint32_t a = colptr[c], b = colptr[c + 1];
    // the reference reads inds[b-1] and inds[a] even for an empty column;
    // reads that would leave [0, nnz) contribute nothing (oracle.c idem)
    if (b == 0 || a >= nnz || b > nnz) continue;
    best = max(best, (inds[b - 1] & kRowMask) - (inds[a] & kRowMask));
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, s));
  if ((threadIdx.x & 63) == 0) atomicMax(result, best);
}

__global__ void __launch_bounds__(kThreads) k_mark(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                   uint32_t nnz, uint32_t rows, const uint32_t* __restrict__ pos,
                                                   uint32_t bit) {
  for (uint64_t e = blockIdx.x * kThreads + threadIdx.x; e < nnz; e += gridDim.x * kThreads) {
    const uint32_t v = in[e], r = v & kRowMask;
    out[e] = r < rows && pos[r] == e ? (v | bit) : v;  // r >= rows was flagged by k_first_last
  }
}

uint32_t grid_for(uint64_t n) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + kThreads - 1) / kThreads, 8192));
}

struct Scratch {  // device buffers freed on every exit path
  void* p[12] = {};
  int n = 0;
  hipEvent_t ev[8] = {};
  hipStream_t s = nullptr;
  ~Scratch() {
    for (int i = 0; i < n; ++i) (void)hipFree(p[i]);
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
  template <typename T>
  hipError_t alloc(T** out, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) p[n++] = q;
    *out = static_cast<T*>(q);
    return e;
  }
};

int fail(hipError_t e, const char* what) {
  set_last_error(std::string(what) + ": " + hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? HIPSPMV_ERR_OOM : HIPSPMV_ERR_HIP;
}

#define PTRY(call)                             \
  do {                                         \
    hipError_t e_ = (call);                    \
    if (e_ != hipSuccess) return fail(e_, #call); \
  } while (0)

float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_device(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_last_error("no HIP device");
    return HIPSPMV_ERR_NO_DEVICE;
  }
  return device < 0 || device >= ndev ? HIPSPMV_ERR_NO_DEVICE : HIPSPMV_OK;
}

}  // namespace

int prep_stats(const uint32_t* colptr, const uint32_t* rowind, uint32_t rows, uint32_t cols, uint32_t nnz,
               int device, hipspmv_prep_stats_t* out) {
  if (!colptr || !out || (nnz && !rowind) || rows == 0 || cols == 0) return HIPSPMV_ERR_INVALID_ARG;
  if (colptr[cols] != nnz) {
    set_last_error("colptr[cols] must equal nnz");
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  if (int st = check_device(device)) return st;
  DevGuard g(device);
  Scratch sc;
  PTRY(hipStreamCreateWithFlags(&sc.s, hipStreamNonBlocking));
  for (auto& e : sc.ev) PTRY(hipEventCreate(&e));
  uint32_t *d_colptr, *d_inds, *d_marked, *d_first, *d_last, *d_res;
  int8_t* d_delta;
  SumMax* d_parts;
  const uint32_t nblk = (uint32_t)(((uint64_t)nnz + kThreads * kItems - 1) / (kThreads * kItems));
  PTRY(sc.alloc(&d_colptr, (size_t)cols + 1));
  PTRY(sc.alloc(&d_inds, nnz));
  PTRY(sc.alloc(&d_marked, nnz));
  PTRY(sc.alloc(&d_first, rows));
  PTRY(sc.alloc(&d_last, rows));
  PTRY(sc.alloc(&d_res, 4));  // [0] bad flag, [1] maxAlive, [2] maxColSpan
  PTRY(sc.alloc(&d_delta, nnz));
  PTRY(sc.alloc(&d_parts, std::max<uint32_t>(nblk, 1)));
  hipStream_t s = sc.s;
  PTRY(hipEventRecord(sc.ev[0], s));
  PTRY(hipMemcpyAsync(d_colptr, colptr, 4ull * (cols + 1), hipMemcpyHostToDevice, s));
  if (nnz) PTRY(hipMemcpyAsync(d_inds, rowind, 4ull * nnz, hipMemcpyHostToDevice, s));
  PTRY(hipMemsetAsync(d_res, 0, 16, s));
  PTRY(hipEventRecord(sc.ev[1], s));
  // maxColSpan
  k_col_span<<<grid_for(cols), kThreads, 0, s>>>(d_colptr, d_inds, cols, nnz, d_res + 2);
  PTRY(hipGetLastError());
  PTRY(hipEventRecord(sc.ev[2], s));
  // maxAlive: first/last positions, delta stream, ordered reduction
  PTRY(hipMemsetAsync(d_first, 0xFF, 4ull * rows, s));
  PTRY(hipMemsetAsync(d_last, 0, 4ull * rows, s));
  PTRY(hipMemsetAsync(d_delta, 0, std::max<size_t>(nnz, 1), s));
  k_first_last<3><<<grid_for(nnz), kThreads, 0, s>>>(d_inds, nnz, rows, d_first, d_last, d_res);
  k_alive_delta<<<grid_for(rows), kThreads, 0, s>>>(d_first, d_last, rows, d_delta);
  if (nblk) {
    k_alive_blocks<<<nblk, kThreads, 0, s>>>(d_delta, nnz, d_parts);
    k_alive_final<<<1, kThreads, 0, s>>>(d_parts, nblk, d_res + 1);
  }
  PTRY(hipGetLastError());
  PTRY(hipEventRecord(sc.ev[3], s));
  // markRowStarts(false, 31) into a scratch copy -- the reference's cmstime
  PTRY(hipMemsetAsync(d_first, 0xFF, 4ull * rows, s));
  k_first_last<1><<<grid_for(nnz), kThreads, 0, s>>>(d_inds, nnz, rows, d_first, d_last, d_res);
  k_mark<<<grid_for(nnz), kThreads, 0, s>>>(d_inds, d_marked, nnz, rows, d_first, 1u << 31);
  PTRY(hipGetLastError());
  PTRY(hipEventRecord(sc.ev[4], s));
  uint32_t res[4] = {0, 0, 0, 0};
  PTRY(hipMemcpyAsync(res, d_res, 16, hipMemcpyDeviceToHost, s));
  PTRY(hipStreamSynchronize(s));
  if (res[0]) {
    set_last_error("row id out of range");
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  out->max_alive = nnz ? res[1] : 0;
  out->max_col_span = res[2];
  out->h2d_ns = (uint64_t)(elapsed(sc.ev[0], sc.ev[1]) * 1e6);
  out->max_col_span_ns = (uint64_t)(elapsed(sc.ev[1], sc.ev[2]) * 1e6);
  out->max_alive_ns = (uint64_t)(elapsed(sc.ev[2], sc.ev[3]) * 1e6);
  out->cms_ns = (uint64_t)(elapsed(sc.ev[3], sc.ev[4]) * 1e6);
  return HIPSPMV_OK;
}

}  // namespace hipspmv

namespace hipspmv {

int mark_row_starts(const uint32_t* rowind, uint32_t* rowind_out, uint32_t rows, uint32_t nnz, int reverse,
                    int shift, int device, uint64_t* kernel_ns) {
  if ((nnz && (!rowind || !rowind_out)) || rows == 0 || shift < 0 || shift > 31) return HIPSPMV_ERR_INVALID_ARG;
  if (int st = check_device(device)) return st;
  if (nnz == 0) {
    if (kernel_ns) *kernel_ns = 0;
    return HIPSPMV_OK;
  }
  DevGuard g(device);
  Scratch sc;
  PTRY(hipStreamCreateWithFlags(&sc.s, hipStreamNonBlocking));
  for (int i = 0; i < 2; ++i) PTRY(hipEventCreate(&sc.ev[i]));
  uint32_t *d_in, *d_out, *d_pos, *d_bad;
  PTRY(sc.alloc(&d_in, nnz));
  PTRY(sc.alloc(&d_out, nnz));
  PTRY(sc.alloc(&d_pos, rows));
  PTRY(sc.alloc(&d_bad, 1));
  hipStream_t s = sc.s;
  PTRY(hipMemcpyAsync(d_in, rowind, 4ull * nnz, hipMemcpyHostToDevice, s));
  PTRY(hipMemsetAsync(d_bad, 0, 4, s));
  PTRY(hipEventRecord(sc.ev[0], s));
  PTRY(hipMemsetAsync(d_pos, reverse ? 0 : 0xFF, 4ull * rows, s));
  if (reverse)
    k_first_last<2><<<grid_for(nnz), kThreads, 0, s>>>(d_in, nnz, rows, d_pos, d_pos, d_bad);
  else
    k_first_last<1><<<grid_for(nnz), kThreads, 0, s>>>(d_in, nnz, rows, d_pos, d_pos, d_bad);
  k_mark<<<grid_for(nnz), kThreads, 0, s>>>(d_in, d_out, nnz, rows, d_pos, 1u << shift);
  PTRY(hipGetLastError());
  PTRY(hipEventRecord(sc.ev[1], s));
  uint32_t bad = 0;
  PTRY(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, s));
  PTRY(hipStreamSynchronize(s));
  if (bad) {
    set_last_error("row id out of range");
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  PTRY(hipMemcpy(rowind_out, d_out, 4ull * nnz, hipMemcpyDeviceToHost));
  if (kernel_ns) *kernel_ns = (uint64_t)(elapsed(sc.ev[0], sc.ev[1]) * 1e6);
  return HIPSPMV_OK;
}

}  // namespace hipspmv
