// layout_probe: does the ORDER in which 256 persistent workgroups stream the
// entry arrays matter?  Each workgroup (1024 threads, one per CU) reads
// `steps` chunks of `chunk` entries (u32 code + 8-byte value each, as the
// vcache layouts store them), a raw barrier per chunk, an 8-deep register
// ring -- the k_vstream entry pipeline without the LDS work.
//   unit-major: workgroup w reads its own contiguous range (chunk s of w at
//               (w * steps + s) * chunk): 256 interleaved sequential streams;
//   step-major: chunk s of w at (s * 256 + w) * chunk: at any moment the chip
//               reads one contiguous window.
// Prints the time of each and the rate over the bytes read.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int kThreads = 1024, kDepth = 8, kEpt = 2;

template <bool STEP_MAJOR>
__global__ __launch_bounds__(kThreads) void k_probe(const uint32_t* __restrict__ code,
                                                    const double* __restrict__ vals, double* __restrict__ out,
                                                    uint32_t steps, uint32_t chunk) {
  const uint32_t w = blockIdx.x, nw = gridDim.x, t = threadIdx.x;
  auto base = [&](uint32_t s) -> size_t {
    const uint32_t sc = s < steps ? s : steps - 1;
    return STEP_MAJOR ? ((size_t)sc * nw + w) * chunk : ((size_t)w * steps + sc) * chunk;
  };
  uint32_t C[kDepth][kEpt];
  double V[kDepth][kEpt];
  auto load = [&](uint32_t s, uint32_t* c, double* v) {
    const size_t b = base(s);
    const uint32_t n = s < steps ? chunk : 0u;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)(code + b), (short)0, (int)(4 * n), 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(vals + b), (short)0, (int)(8 * n), 0x00020000);
#pragma unroll
    for (int j = 0; j < kEpt; ++j) {
      c[j] = __builtin_amdgcn_raw_buffer_load_b32(rc, 4 * (t + j * kThreads), 0, 0);
      v[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rv, 8 * (t + j * kThreads), 0, 0));
    }
  };
  double acc = 0.0;
#pragma unroll
  for (int d = 0; d < kDepth; ++d) load(d, C[d], V[d]);
  const uint32_t nsteps = (steps + kDepth - 1) / kDepth * kDepth;
  for (uint32_t b0 = 0; b0 < nsteps; b0 += kDepth) {
#pragma unroll
    for (int i = 0; i < kDepth; ++i) {
#pragma unroll
      for (int j = 0; j < kEpt; ++j) acc += (double)C[i][j] + V[i][j];
      load(b0 + i + kDepth, C[i], V[i]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  out[(size_t)w * kThreads + t] = acc;
}

int main() {
  const uint32_t nw = 256, chunk = 1000, steps = 131;  // ~ the C3 split4 unit: 131k entries per CU
  const size_t n = (size_t)nw * steps * chunk;
  uint32_t* code;
  double *vals, *out;
  CK(hipMalloc(&code, 4 * n));
  CK(hipMalloc(&vals, 8 * n));
  CK(hipMalloc(&out, 8ull * nw * kThreads));
  CK(hipMemset(code, 1, 4 * n));
  CK(hipMemset(vals, 0, 8 * n));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rnd = 0; rnd < 2; ++rnd) {
    for (int sm = 0; sm < 2; ++sm) {
      auto launch = [&] {
        if (sm)
          hipLaunchKernelGGL(k_probe<true>, dim3(nw), dim3(kThreads), 0, 0, code, vals, out, steps, chunk);
        else
          hipLaunchKernelGGL(k_probe<false>, dim3(nw), dim3(kThreads), 0, 0, code, vals, out, steps, chunk);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipEventRecord(e0, 0));
      const int reps = 20;
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      std::printf("%s: %8.2f us  %7.1f GB/s (%zu entries, 12 B each)\n", sm ? "step-major" : "unit-major", us,
                  12.0 * n / us / 1e3, n);
    }
  }
  return 0;
}
