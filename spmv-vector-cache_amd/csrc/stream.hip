// The measured HBM ceiling beside the roofline's 8 TB/s (SURVEY.md §8(d)'s
// second denominator): a streaming copy and a streaming
// read of buffers far larger than the 256 MiB Infinity Cache, 16-byte
// non-temporal accesses, grid-stride with four loads in flight per lane before
// their stores -- the access pattern MI355X_MICROARCH.md quotes ~6.3 TB/s for.
// Not on the SpMV path: hipspmv_stream_bandwidth is what bench.py reports as
// `measured_copy_gbs` / `measured_read_gbs`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "hipspmv.h"
#include "hipspmv_internal.h"

namespace hipspmv {

namespace {

typedef unsigned int u32x4s __attribute__((ext_vector_type(4)));
constexpr int kStT = 256, kStU = 4;  // threads per block, 16-byte loads in flight per lane

__global__ __launch_bounds__(kStT) void k_stream_copy(const u32x4s* __restrict__ src, u32x4s* __restrict__ dst,
                                                      uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * kStT * kStU;
  for (uint64_t b = (uint64_t)blockIdx.x * kStT * kStU + threadIdx.x; b < n; b += stride) {
    u32x4s v[kStU];
#pragma unroll
    for (int k = 0; k < kStU; ++k)
      if (b + (uint64_t)k * kStT < n) v[k] = __builtin_nontemporal_load(src + b + (uint64_t)k * kStT);
#pragma unroll
    for (int k = 0; k < kStU; ++k)
      if (b + (uint64_t)k * kStT < n) __builtin_nontemporal_store(v[k], dst + b + (uint64_t)k * kStT);
  }
}

// reads every byte once; one store per lane keeps the loads alive
__global__ __launch_bounds__(kStT) void k_stream_read(const u32x4s* __restrict__ src, uint64_t n,
                                                      unsigned* __restrict__ sink) {
  const uint64_t stride = (uint64_t)gridDim.x * kStT * kStU;
  unsigned acc = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * kStT * kStU + threadIdx.x; b < n; b += stride) {
    u32x4s v[kStU];
#pragma unroll
    for (int k = 0; k < kStU; ++k)
      v[k] = b + (uint64_t)k * kStT < n ? __builtin_nontemporal_load(src + b + (uint64_t)k * kStT) : u32x4s{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < kStU; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  sink[(uint64_t)blockIdx.x * kStT + threadIdx.x] = acc;
}

}  // namespace

}  // namespace hipspmv

using namespace hipspmv;

extern "C" int hipspmv_stream_bandwidth(int device, uint64_t bytes, int reps, double* copy_gbs, double* read_gbs) {
  if (bytes < (1u << 20) || reps < 1 || (!copy_gbs && !read_gbs)) return HIPSPMV_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return HIPSPMV_ERR_NO_DEVICE;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  const uint64_t n = bytes / 16;
  const int blocks = 2048;  // 8 per CU on 256 CUs: 2048 threads per CU
  u32x4s *a = nullptr, *b = nullptr;
  unsigned* sink = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int st = HIPSPMV_OK;
  auto fail = [&](hipError_t e) {
    set_last_error(std::string("hipspmv_stream_bandwidth: ") + hipGetErrorString(e));
    st = e == hipErrorOutOfMemory ? HIPSPMV_ERR_OOM : HIPSPMV_ERR_HIP;
  };
  hipError_t e = hipMalloc(&a, 16 * n);
  if (e == hipSuccess) e = hipMalloc(&b, 16 * n);
  if (e == hipSuccess) e = hipMalloc(&sink, sizeof(unsigned) * blocks * kStT);
  if (e == hipSuccess) e = hipMemset(a, 1, 16 * n);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  auto timed = [&](auto launch) -> double {  // ms per launch after two untimed ones
    for (int i = 0; i < 2; ++i) launch();
    if ((e = hipEventRecord(e0, nullptr)) != hipSuccess) return 0;
    for (int i = 0; i < reps; ++i) launch();
    if ((e = hipEventRecord(e1, nullptr)) != hipSuccess || (e = hipEventSynchronize(e1)) != hipSuccess) return 0;
    float ms = 0;
    e = hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
  };
  if (e == hipSuccess && copy_gbs) {
    const double ms = timed([&] { hipLaunchKernelGGL(k_stream_copy, dim3(blocks), dim3(kStT), 0, nullptr, a, b, n); });
    if (e == hipSuccess) e = hipGetLastError();
    *copy_gbs = e == hipSuccess && ms > 0 ? 2.0 * 16 * n / (ms * 1e-3) / 1e9 : 0.0;
  }
  if (e == hipSuccess && read_gbs) {
    const double ms = timed([&] { hipLaunchKernelGGL(k_stream_read, dim3(blocks), dim3(kStT), 0, nullptr, a, n, sink); });
    if (e == hipSuccess) e = hipGetLastError();
    *read_gbs = e == hipSuccess && ms > 0 ? 16.0 * n / (ms * 1e-3) / 1e9 : 0.0;
  }
  if (e != hipSuccess) fail(e);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (sink) (void)hipFree(sink);
  if (prev >= 0) (void)hipSetDevice(prev);
  return st;
}
