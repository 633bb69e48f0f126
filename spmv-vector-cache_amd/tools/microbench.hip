// Design-space microbenchmark for the HIPSpMV hot path on gfx950 (MI355X).
//
// Not product code: a standalone probe, run once per design question, that
// times candidate inner loops of the SpMV row gather on the C3 workload
// (2^20 x 2^20, 32 nnz/row, one column per 2^15-wide stripe)
// generated on the device, so that kernel structure is chosen from
// measurements rather than guesses.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o microbench microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__host__ __device__ inline uint64_t sm64(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline double u11(uint64_t z) { return (double)(z >> 11) * 0x1.0p-52 - 1.0; }

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef uint32_t uv4 __attribute__((ext_vector_type(4)));
typedef uint32_t uv2 __attribute__((ext_vector_type(2)));

constexpr int LOGN = 20;
constexpr uint32_t N = 1u << LOGN;
constexpr int K = 32;
constexpr uint32_t STRIPE = N / K;
constexpr uint64_t NNZ = (uint64_t)N * K;

__global__ void gen_csr(uint32_t* rowptr, uint32_t* col, double* val, double* x) {
  uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e < NNZ) {
    uint32_t k = e % K;
    col[e] = k * STRIPE + (uint32_t)(sm64(1, e) % STRIPE);
    val[e] = u11(sm64(2, e));
  }
  if (e <= N) rowptr[e] = (uint32_t)(e * K);
  if (e < N) x[e] = u11(sm64(3, e));
}
// SELL-64: [slice][k][lane]
__global__ void gen_sell(const uint32_t* col, const double* val, uint32_t* scol, double* sval) {
  uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e >= NNZ) return;
  uint64_t r = e / K, k = e % K;
  uint64_t d = (r / 64) * 64 * K + k * 64 + (r % 64);
  scol[d] = col[e]; sval[d] = val[e];
}
// SELL-64 with 16-byte lanes: vals in pairs [slice][k/2][lane][2], cols in quads [slice][k/4][lane][4]
__global__ void gen_sell2(const uint32_t* col, const double* val, uint32_t* scol, double* sval) {
  uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (e >= NNZ) return;
  uint64_t r = e / K, k = e % K, s = r / 64, l = r % 64;
  sval[s * 64 * K + (k / 2) * 128 + l * 2 + (k & 1)] = val[e];
  scol[s * 64 * K + (k / 4) * 256 + l * 4 + (k & 3)] = col[e];
}

__global__ void k_copy(const dv2* __restrict__ a, dv2* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = __builtin_nontemporal_load(&a[i]);
}

template <typename T, bool NT> __device__ inline T ld(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}

// lane-per-row, ordered (sequential per row, no FMA): NS slices per wave
template <int NS, bool NT>
__global__ __launch_bounds__(256) void k_sell_lane(const uint32_t* __restrict__ scol, const double* __restrict__ sval,
                                                    const double* __restrict__ x, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t s0 = wave * NS;
  double acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = 0.0;
#pragma unroll 4
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      size_t idx = (size_t)(s0 + s) * 64 * K + k * 64 + lane;
      uint32_t c = ld<uint32_t, NT>(&scol[idx]);
      double v = ld<double, NT>(&sval[idx]);
      acc[s] = acc[s] + v * x[c];
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) y[(size_t)(s0 + s) * 64 + lane] = acc[s];
}

// lane-per-row with 16-byte loads (gen_sell2 layout)
template <bool NT>
__global__ __launch_bounds__(256) void k_sell_lane16(const uint32_t* __restrict__ scol, const double* __restrict__ sval,
                                                      const double* __restrict__ x, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const uint32_t s0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const dv2* v2 = reinterpret_cast<const dv2*>(sval + (size_t)s0 * 64 * K);
  const uv4* c4 = reinterpret_cast<const uv4*>(scol + (size_t)s0 * 64 * K);
  double acc = 0.0;
#pragma unroll 2
  for (int k4 = 0; k4 < K / 4; ++k4) {
    uv4 c = ld<uv4, NT>(&c4[k4 * 64 + lane]);
    dv2 va = ld<dv2, NT>(&v2[(2 * k4) * 64 + lane]);
    dv2 vb = ld<dv2, NT>(&v2[(2 * k4 + 1) * 64 + lane]);
    double x0 = x[c.x], x1 = x[c.y], x2 = x[c.z], x3 = x[c.w];
    acc = acc + va.x * x0; acc = acc + va.y * x1; acc = acc + vb.x * x2; acc = acc + vb.y * x3;
  }
  y[(size_t)s0 * 64 + lane] = acc;
}

template <int CTRL> __device__ inline double dpp(double v) {
  int2 t = __builtin_bit_cast(int2, v);
  t.x = __builtin_amdgcn_mov_dpp(t.x, CTRL, 0xF, 0xF, false);
  t.y = __builtin_amdgcn_mov_dpp(t.y, CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, t);
}

// CSR, 16 lanes per row, 2 elements per lane (16-byte value loads), DPP row reduce
template <bool NT>
__global__ __launch_bounds__(256) void k_csr_sub16(const uint32_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                                    const double* __restrict__ val, const double* __restrict__ x,
                                                    double* __restrict__ y, uint32_t rows_per_wave) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t r0 = wave * rows_per_wave;
  for (uint32_t rr = 0; rr < rows_per_wave; rr += 4) {
    uint32_t r = r0 + rr + (lane >> 4);
    uint32_t b = rowptr[r];
    uint32_t e = b + 2 * (lane & 15);
    dv2 v = ld<dv2, NT>(reinterpret_cast<const dv2*>(val + e));
    uv2 c = ld<uv2, NT>(reinterpret_cast<const uv2*>(col + e));
    double s = v.x * x[c.x] + v.y * x[c.y];
    s += dpp<0xB1>(s);
    s += dpp<0x4E>(s);
    s += dpp<0x124>(s);
    s += dpp<0x128>(s);
    if ((lane & 15) == 0) y[r] = s;
  }
}

// gather-only: 32 gathers per lane into an x of 2^xbits doubles, stripe pattern, hashed indices
__global__ __launch_bounds__(256) void k_gather(const double* __restrict__ x, double* __restrict__ y, int xbits) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stripe = (1u << xbits) / K;
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    uint32_t h = (uint32_t)sm64(7, (uint64_t)r * K + k);
    acc += x[k * stripe + (h & (stripe - 1))];
  }
  y[r] = acc;
}

// stream-only: read SELL vals/cols, no gather
template <bool NT>
__global__ __launch_bounds__(256) void k_stream(const uint32_t* __restrict__ scol, const double* __restrict__ sval,
                                                 double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const uint32_t s0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  double acc = 0.0;
#pragma unroll 8
  for (int k = 0; k < K; ++k) {
    size_t idx = (size_t)s0 * 64 * K + k * 64 + lane;
    acc += ld<double, NT>(&sval[idx]) + (double)ld<uint32_t, NT>(&scol[idx]);
  }
  y[(size_t)s0 * 64 + lane] = acc;
}


// ---------------------------------------------------------------------------
// "vector cache" kernel: one workgroup per row block (<= VR rows, y kept in LDS),
// x streamed through LDS in panels of VP columns (double-buffered, register-staged
// one panel ahead), entries stored per (block, panel) segment sorted by (row, col).
// Entry code: col_local[0:16) | row_local[16:30) | CONT(bit30) | MORE(bit31).
constexpr int VT = 1024, VP = 8192, VR = 4096, EPT = 2;
constexpr uint32_t CONT = 1u << 30, MORE = 1u << 31;

template <bool NT>
__global__ __launch_bounds__(1024) void k_vcache(const uint32_t* __restrict__ seg, const uint32_t* __restrict__ eidx,
                                                  const double* __restrict__ evals, const double* __restrict__ x,
                                                  double* __restrict__ y, uint32_t cols, uint32_t npanels, uint32_t last) {
  __shared__ double ylds[VR];
  __shared__ double xb[2][VP];
  const int t = threadIdx.x;
  const uint32_t b = blockIdx.x;
  for (int i = t; i < VR; i += VT) ylds[i] = 0.0;
  const uint32_t* sp = seg + (size_t)b * npanels;
  // x panel loads: branch-free, clamped to the last in-bounds 16-byte pair; for odd cols the
  // final element is patched from a scalar load by the thread that owns its LDS slot.
  const uint32_t cmax = (cols - 2) & ~1u;
  const double xlast = x[cols - 1];
  auto load_x = [&](uint32_t p, dv2* r) {
    const uint32_t base = min(p, npanels - 1) * VP;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const dv2*>(x + min(base + 2 * (t + j * VT), cmax));
  };
  auto store_x = [&](uint32_t p, const dv2* r) {
    double* dst = xb[p & 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<dv2*>(&dst[2 * (t + j * VT)]) = r[j];
    if ((cols & 1) && p == npanels - 1) {
      uint32_t slot = cols - 1 - p * VP;
      if (t == (slot >> 1) % VT) dst[slot] = xlast;
    }
  };
  auto load_e = [&](uint32_t p, uint32_t* c, double* v) {  // branch-free: clamped index, validity checked at use
    uint32_t beg = sp[min(p, npanels - 1)];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      uint32_t i = min(beg + t + j * VT, last);
      c[j] = ld<uint32_t, NT>(eidx + i); v[j] = ld<double, NT>(evals + i);
    }
  };
  auto run = [&](uint32_t i, uint32_t code, double v, const double* xs) {
    uint32_t row = (code >> 16) & 0x3FFF;
    double acc = ylds[row];
    acc = acc + v * xs[code & 0xFFFF];
    while (code & MORE) { ++i; code = eidx[i]; acc = acc + evals[i] * xs[code & 0xFFFF]; }
    ylds[row] = acc;
  };
  dv2 xa[4], xb2[4];
  uint32_t eca[EPT], ecb[EPT]; double eva[EPT], evb[EPT];
  load_x(0, xa); store_x(0, xa);
  load_x(1, xa);
  load_e(0, eca, eva);
  __syncthreads();
  // one panel step: consume (cc, cv, xcur) for panel p, prefetch panel p+1 entries into (nc, nv) and panel p+2 x into xnext
  auto step = [&](uint32_t p, uint32_t* cc, double* cv, dv2* xcur, uint32_t* nc, double* nv, dv2* xnext) {
    load_e(p + 1, nc, nv);
    load_x(p + 2, xnext);
    const double* xs = xb[p & 1];
    const uint32_t beg = sp[p], end = sp[p + 1];
#pragma unroll
    for (int j = 0; j < EPT; ++j)
      if (beg + t + j * VT < end && !(cc[j] & CONT)) run(beg + t + j * VT, cc[j], cv[j], xs);
    for (uint32_t i = beg + EPT * VT + t; i < end; i += VT) {
      uint32_t code = eidx[i];
      if (!(code & CONT)) run(i, code, evals[i], xs);
    }
    if (p + 1 < npanels) store_x(p + 1, xcur);
    __syncthreads();
  };
  uint32_t p = 0;
  for (; p + 1 < npanels; p += 2) {
    step(p, eca, eva, xa, ecb, evb, xb2);
    step(p + 1, ecb, evb, xb2, eca, eva, xa);
  }
  if (p < npanels) step(p, eca, eva, xa, ecb, evb, xb2);
  for (int i = t; i < VR; i += VT) y[(size_t)b * VR + i] = ylds[i];
}

// depth-D pipelined variant: entries and x panels both prefetched D panels ahead in
// register rings (statically indexed by full unroll), LDS holds y + 2 x buffers.
template <int D, bool NT>
__global__ __launch_bounds__(1024) void k_vcacheD(const uint32_t* __restrict__ seg, const uint32_t* __restrict__ eidx,
                                                   const double* __restrict__ evals, const double* __restrict__ x,
                                                   double* __restrict__ y, uint32_t cols, uint32_t npanels,
                                                   uint32_t npad, uint32_t last, uint32_t ablate = 0) {
  __shared__ double ylds[VR];
  __shared__ double xb[2][VP];
  const int t = threadIdx.x;
  const uint32_t b = blockIdx.x;
  for (int i = t; i < VR; i += VT) ylds[i] = 0.0;
  const uint32_t* sp = seg + (size_t)b * (npad + 1);
  const uint32_t cmax = (cols - 2) & ~1u;
  const double xlast = x[cols - 1];
  dv2 X[D][4] = {};
  uint32_t EC[D][EPT] = {}; double EV[D][EPT] = {};
  auto load_x = [&](uint32_t p, dv2* r) {
    if (ablate & 2) return;
    const uint32_t base = (ablate & 1) ? 0 : min(p, npanels - 1) * VP;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const dv2*>(x + min(base + 2 * (t + j * VT), cmax));
  };
  auto store_x = [&](uint32_t p, const dv2* r) {
    double* dst = xb[p & 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<dv2*>(&dst[2 * (t + j * VT)]) = r[j];
    if ((cols & 1) && p == npanels - 1) {
      uint32_t slot = cols - 1 - p * VP;
      if (t == (slot >> 1) % VT) dst[slot] = xlast;
    }
  };
  auto load_e = [&](uint32_t p, uint32_t* c, double* v) {
    if (ablate & 8) return;
    uint32_t beg = sp[min(p, npad)];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      uint32_t i = min(beg + t + j * VT, last);
      c[j] = ld<uint32_t, NT>(eidx + i); v[j] = ld<double, NT>(evals + i);
    }
  };
  auto run = [&](uint32_t i, uint32_t code, double v, const double* xs) {
    uint32_t row = (code >> 16) & 0x3FFF;
    double acc = ylds[row];
    acc = acc + v * xs[code & 0xFFFF];
    while (code & MORE) { ++i; code = eidx[i]; acc = acc + evals[i] * xs[code & 0xFFFF]; }
    ylds[row] = acc;
  };
  // prologue: x(0) -> LDS; X ring holds x(1..D), E ring holds entries(0..D-1)
  load_x(0, X[0]); store_x(0, X[0]);
#pragma unroll
  for (int i = 0; i < D; ++i) { load_e(i, EC[i], EV[i]); load_x(i + 1, X[(i + 1) % D]); }
  __syncthreads();
  for (uint32_t base = 0; base < npad; base += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const uint32_t s = base + i;
      const double* xs = xb[s & 1];
      const uint32_t beg = sp[s], end = sp[s + 1];
#pragma unroll
      for (int j = 0; j < EPT; ++j)
        if (!(ablate & 4) && beg + t + j * VT < end && !(EC[i][j] & CONT)) run(beg + t + j * VT, EC[i][j], EV[i][j], xs);
      if (!(ablate & 4)) for (uint32_t q = beg + EPT * VT + t; q < end; q += VT) {
        uint32_t code = eidx[q];
        if (!(code & CONT)) run(q, code, evals[q], xs);
      }
      load_e(s + D, EC[i], EV[i]);
      store_x(s + 1, X[(i + 1) % D]);
      load_x(s + 1 + D, X[(i + 1) % D]);
      __syncthreads();
    }
  }
  for (int i = t; i < VR; i += VT) y[(size_t)b * VR + i] = ylds[i];
}

template <typename F> double time_us(F f, int reps = 30) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) f();
  std::vector<float> t;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1000.f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const double algB = 12.0 * NNZ + 4.0 * (N + 1) + 8.0 * N + 8.0 * N;
  uint32_t *rowptr, *col, *scol, *scol2; double *val, *sval, *sval2, *x, *y, *y2;
  CK(hipMalloc(&rowptr, 4ull * (N + 1))); CK(hipMalloc(&col, 4 * NNZ)); CK(hipMalloc(&val, 8 * NNZ));
  CK(hipMalloc(&scol, 4 * NNZ)); CK(hipMalloc(&sval, 8 * NNZ));
  CK(hipMalloc(&scol2, 4 * NNZ)); CK(hipMalloc(&sval2, 8 * NNZ));
  CK(hipMalloc(&x, 8ull << 28)); CK(hipMalloc(&y, 8ull * N)); CK(hipMalloc(&y2, 8ull * N));
  gen_csr<<<(NNZ + 255) / 256, 256>>>(rowptr, col, val, x);
  gen_sell<<<(NNZ + 255) / 256, 256>>>(col, val, scol, sval);
  gen_sell2<<<(NNZ + 255) / 256, 256>>>(col, val, scol2, sval2);
  CK(hipDeviceSynchronize());

  // host reference for row 12345 and a checksum
  auto check = [&](const char* name) {
    std::vector<double> h(N), hr(N);
    CK(hipMemcpy(h.data(), y, 8ull * N, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), y2, 8ull * N, hipMemcpyDeviceToHost));
    double md = 0; for (uint32_t i = 0; i < N; ++i) md = std::max(md, std::fabs(h[i] - hr[i]));
    printf("   [%s] max|diff| vs sell_lane ref = %.3e\n", name, md);
  };
  // reference y2 via NS=1 sell lane
  k_sell_lane<1, false><<<N / 256, 256>>>(scol, sval, x, y2);
  CK(hipDeviceSynchronize());

  auto report = [&](const char* name, double us) {
    printf("%-34s %9.2f us  %8.1f GB/s(alg)  %7.1f GFLOP/s  frac8TB=%.3f\n", name, us, algB / us * 1e-3,
           2.0 * NNZ / us * 1e-3, algB / us * 1e-3 / 8000.0);
  };

  {
    size_t n2 = (512ull << 20) / 16;
    double us = time_us([&] { k_copy<<<8192, 256>>>((const dv2*)x, (dv2*)(x + (512ull << 20) / 8 / 2 * 0 + (1ull << 27)), n2 / 2); });
    printf("%-34s %9.2f us  %8.1f GB/s (256MB read + 256MB write)\n", "copy 2x256MB", us, 512.0 * 1048576 / us * 1e-3);
  }
  report("stream-only sell (plain)", time_us([&] { k_stream<false><<<N / 256, 256>>>(scol, sval, y); }));
  report("stream-only sell (nt)", time_us([&] { k_stream<true><<<N / 256, 256>>>(scol, sval, y); }));
  for (int xb = 17; xb <= 26; ++xb) {
    double us = time_us([&] { k_gather<<<N / 256, 256>>>(x, y, xb); });
    printf("gather-only x=2^%d doubles (%6.1f MB)  %9.2f us  %7.2f Ggather/s\n", xb, 8.0 * (1 << xb) / 1048576, us,
           NNZ / us * 1e-3);
  }
  report("sell_lane NS=1", time_us([&] { k_sell_lane<1, false><<<N / 256, 256>>>(scol, sval, x, y); })); check("NS1");
  report("sell_lane NS=1 nt", time_us([&] { k_sell_lane<1, true><<<N / 256, 256>>>(scol, sval, x, y); })); check("NS1nt");
  report("sell_lane NS=2 nt", time_us([&] { k_sell_lane<2, true><<<N / 512, 256>>>(scol, sval, x, y); })); check("NS2");
  report("sell_lane NS=4 nt", time_us([&] { k_sell_lane<4, true><<<N / 1024, 256>>>(scol, sval, x, y); })); check("NS4");
  report("sell_lane NS=8 nt", time_us([&] { k_sell_lane<8, true><<<N / 2048, 256>>>(scol, sval, x, y); })); check("NS8");
  report("sell_lane16 plain", time_us([&] { k_sell_lane16<false><<<N / 256, 256>>>(scol2, sval2, x, y); })); check("L16");
  report("sell_lane16 nt", time_us([&] { k_sell_lane16<true><<<N / 256, 256>>>(scol2, sval2, x, y); })); check("L16nt");
  for (uint32_t rpw : {4u, 16u, 64u}) {
    char nm[64]; snprintf(nm, sizeof nm, "csr_sub16 rpw=%u nt", rpw);
    report(nm, time_us([&] { k_csr_sub16<true><<<N / rpw / 4, 256>>>(rowptr, col, val, x, y, rpw); })); check(nm);
  }
  report("csr_sub16 rpw=16 plain", time_us([&] { k_csr_sub16<false><<<N / 16 / 4, 256>>>(rowptr, col, val, x, y, 16); }));

  {
    // host build of the (block, panel) segment layout from the C3 generator
    const uint32_t NB = N / VR, NPAN = (N + VP - 1) / VP;
    std::vector<uint32_t> cnt((size_t)NB * NPAN + 1, 0);
    std::vector<uint32_t> hc(NNZ);
    for (uint64_t e = 0; e < NNZ; ++e) hc[e] = (uint32_t)(e % K) * STRIPE + (uint32_t)(sm64(1, e) % STRIPE);
    for (uint64_t e = 0; e < NNZ; ++e) { uint32_t r = e / K; cnt[(size_t)(r / VR) * NPAN + hc[e] / VP + 1]++; }
    for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
    std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1), code(NNZ);
    std::vector<double> hv(NNZ);
    std::vector<uint32_t> lastrow((size_t)NB * NPAN, 0xFFFFFFFF);
    for (uint64_t e = 0; e < NNZ; ++e) {
      uint32_t r = e / K, c = hc[e];
      size_t key = (size_t)(r / VR) * NPAN + c / VP;
      uint32_t d = pos[key]++;
      uint32_t cd = (c % VP) | ((r % VR) << 16);
      if (lastrow[key] == r) { cd |= CONT; code[d - 1] |= MORE; }
      lastrow[key] = r;
      code[d] = cd; hv[d] = u11(sm64(2, e));
    }
    uint32_t maxseg = 0; for (size_t i = 0; i + 1 < cnt.size(); ++i) maxseg = std::max(maxseg, cnt[i + 1] - cnt[i]);
    printf("vcache layout: %u blocks x %u panels, max seg %u entries\n", NB, NPAN, maxseg);
    uint32_t *dseg, *dcode; double* dval;
    CK(hipMalloc(&dseg, 4 * cnt.size())); CK(hipMalloc(&dcode, 4 * NNZ)); CK(hipMalloc(&dval, 8 * NNZ));
    CK(hipMemcpy(dseg, cnt.data(), 4 * cnt.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dcode, code.data(), 4 * NNZ, hipMemcpyHostToDevice));
    CK(hipMemcpy(dval, hv.data(), 8 * NNZ, hipMemcpyHostToDevice));
    report("vcache nt", time_us([&] { k_vcache<true><<<NB, VT>>>(dseg, dcode, dval, x, y, N, NPAN, (uint32_t)NNZ - 1); })); check("vcache nt");
    report("vcache plain", time_us([&] { k_vcache<false><<<NB, VT>>>(dseg, dcode, dval, x, y, N, NPAN, (uint32_t)NNZ - 1); })); check("vcache");


    {
      uint32_t npad = (NPAN + 2) / 3 * 3;
      std::vector<uint32_t> segp((size_t)NB * (npad + 1));
      for (uint32_t bb = 0; bb < NB; ++bb)
        for (uint32_t pp = 0; pp <= npad; ++pp) segp[(size_t)bb * (npad + 1) + pp] = cnt[(size_t)bb * NPAN + std::min(pp, NPAN)];
      uint32_t* dsegp; CK(hipMalloc(&dsegp, 4 * segp.size()));
      CK(hipMemcpy(dsegp, segp.data(), 4 * segp.size(), hipMemcpyHostToDevice));
      const char* names[] = {"full", "x from panel0 (L2)", "no x loads", "", "no compute", "no compute, x panel0", "no compute, no x", "", "no entry loads", "", "no entries, no x"};
      for (uint32_t ab : {0u, 1u, 2u, 4u, 5u, 6u, 8u, 10u}) {
        char nm[64]; snprintf(nm, sizeof nm, "ablate D=3: %s", names[ab]);
        report(nm, time_us([&] { k_vcacheD<3, false><<<NB, VT>>>(dsegp, dcode, dval, x, y, N, NPAN, npad, (uint32_t)NNZ - 1, ab); }));
      }
      CK(hipFree(dsegp));
    }
    for (int D : {2, 3, 4}) {
      // padded segment table: per block npad+1 offsets, npad = npanels rounded up to D
      uint32_t npad = (NPAN + D - 1) / D * D;
      std::vector<uint32_t> segp((size_t)NB * (npad + 1));
      for (uint32_t bb = 0; bb < NB; ++bb)
        for (uint32_t pp = 0; pp <= npad; ++pp) segp[(size_t)bb * (npad + 1) + pp] = cnt[(size_t)bb * NPAN + std::min(pp, NPAN)];
      uint32_t* dsegp; CK(hipMalloc(&dsegp, 4 * segp.size()));
      CK(hipMemcpy(dsegp, segp.data(), 4 * segp.size(), hipMemcpyHostToDevice));
      char nm[64];
      auto go = [&](auto kern) { return time_us([&] { kern<<<NB, VT>>>(dsegp, dcode, dval, x, y, N, NPAN, npad, (uint32_t)NNZ - 1, 0u); }); };
      snprintf(nm, sizeof nm, "vcacheD D=%d nt", D);
      if (D == 2) report(nm, go(k_vcacheD<2, true>)); if (D == 3) report(nm, go(k_vcacheD<3, true>)); if (D == 4) report(nm, go(k_vcacheD<4, true>));
      check(nm);
      snprintf(nm, sizeof nm, "vcacheD D=%d plain", D);
      if (D == 2) report(nm, go(k_vcacheD<2, false>)); if (D == 3) report(nm, go(k_vcacheD<3, false>)); if (D == 4) report(nm, go(k_vcacheD<4, false>));
      check(nm);
      CK(hipFree(dsegp));
    }
    {
      std::vector<double> h(N), hr(N);
      CK(hipMemcpy(h.data(), y, 8ull * N, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hr.data(), y2, 8ull * N, hipMemcpyDeviceToHost));
      printf("   vcache bitwise equal to sell_lane: %s\n", memcmp(h.data(), hr.data(), 8ull * N) == 0 ? "yes" : "NO");
    }
  }
  return 0;
}
