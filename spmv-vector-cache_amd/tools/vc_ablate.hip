// Diagnostic build of k_vcache (csrc/vcache.hip): times the kernel on config
// C3 for several (loader waves, entry depth, entries/lane) settings and with
// parts of its work ablated (AB template mask), to attribute its time.
// Results are wrong by construction except for mask 0; only timings matter.
// Not part of the product libraries.
//
//   make -C spmv-vector-cache_amd lib/vc_ablate && ./spmv-vector-cache_amd/lib/vc_ablate
#include "../csrc/vcache.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../host/Synthetic.h"

using namespace hipspmv;

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__);  \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

template <typename T>
T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, sizeof(T) * std::max<size_t>(v.size(), 1)));
  CK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const uint32_t n = 1u << (argc > 1 ? std::atoi(argv[1]) : 20), k = 32;
  HostCSR a;
  a.rows = a.cols = n;
  a.nnz = n * k;
  a.rowptr.resize(n + 1);
  a.colind.resize(a.nnz);
  std::vector<double> v(a.nnz);
  genStripeCSR(0, n, n, k, 1, 2, a.rowptr.data(), a.colind.data(), v.data());
  a.vals.assign(reinterpret_cast<uint64_t*>(v.data()), reinterpret_cast<uint64_t*>(v.data()) + a.nnz);
  std::vector<double> x(n);
  for (uint32_t i = 0; i < n; ++i) x[i] = uniform11(splitmix64_at(3, i));
  double* dx = up(x);
  double *dy, *dpart;
  CK(hipMalloc(&dy, 8ull * n));
  CK(hipMalloc(&dpart, 16ull * n));
  const double alg = 12.0 * a.nnz + 4.0 * (n + 1) + 16.0 * n;
  auto timeit = [&](auto launch) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) launch();
    std::vector<float> ts;
    for (int r = 0; r < 15; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
  };
  std::vector<double> yref;
  for (VcGeom g : {kVcOrdered, kVcSplit}) {
    VcacheLayout L;
    build_vcache(a, g, L);
    VcacheArgs A{up(L.seg), up(L.code), up(L.vals), dx, dy, dy, dpart, up(std::vector<uint32_t>(L.nblocks, 0)),
                 a.rows, a.cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels, L.npad, a.nnz - 1,
                 g.split, 0};
    std::printf("geometry rows=%d panel=%d split=%d: units=%u npad=%u max_seg=%u\n", g.rows, g.panel, g.split,
                L.nblocks * g.split, L.npad, L.max_seg);
    auto variant = [&](auto kern, const char* nm, int mask) {
      const double us = timeit([&] {
        hipLaunchKernelGGL(kern, dim3(A.nblocks * A.split), dim3(kVcThreads), 0, nullptr, A.seg, A.code,
                           (const double*)A.vals, (const double*)A.x, (const double*)A.y_in, (double*)A.y_out,
                           (double*)A.partial, A.tickets, A.rows, A.cols, A.rows_per_block, A.nblocks, A.npanels,
                           A.part_panels, A.npad, A.last, A.beta);
      });
      std::printf("  %-30s mask %2d %8.2f us  (alg %6.1f GB/s)", nm, mask, us, alg / us * 1e-3);
      if (mask == 0) {  // compare against the first (ordered) result
        std::vector<double> y(n);
        CK(hipMemcpy(y.data(), dy, 8ull * n, hipMemcpyDeviceToHost));
        if (yref.empty()) yref = y;
        double md = 0;
        for (uint32_t i = 0; i < n; ++i) md = std::max(md, std::abs(y[i] - yref[i]));
        std::printf("  max|y-y_ordered|=%.2e", md);
      }
      std::printf("\n");
    };
    if (g.split == 1) {
      variant(k_vcache<double, 1>, "default (WL8 DE4 EPT3)", 0);
      variant(k_vcache<double, 1, 4, 4, 2>, "WL4 DE4 EPT2", 0);
      variant(k_vcache<double, 1, 8, 2, 3>, "WL8 DE2 EPT3", 0);
      variant(k_vcache<double, 1, 8, 6, 3>, "WL8 DE6 EPT3", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 3>, "no x", 3);
      variant(k_vcache<double, 1, 8, 4, 3, 12>, "no entries/compute", 12);
      variant(k_vcache<double, 1, 8, 4, 3, 15>, "skeleton", 15);
    } else {
      variant(k_vcache<double, 2>, "default (WL4 DE4 EPT3)", 0);
      variant(k_vcache<double, 2, 4, 2, 3>, "WL4 DE2 EPT3", 0);
      variant(k_vcache<double, 2, 4, 6, 3>, "WL4 DE6 EPT3", 0);
      variant(k_vcache<double, 2, 6, 4, 3>, "WL6 DE4 EPT3", 0);
      variant(k_vcache<double, 2, 8, 4, 4>, "WL8 DE4 EPT4", 0);
      variant(k_vcache<double, 2, 6, 4, 3, 0, 1, false>, "WL6 MAP1", 0);
      variant(k_vcache<double, 2, 6, 4, 3, 0, 0, true>, "WL6 NT", 0);
      variant(k_vcache<double, 2, 6, 4, 3, 0, 1, true>, "WL6 MAP1 NT", 0);
      variant(k_vcache<double, 2, 6, 4, 3, 16, 1, true>, "WL6 MAP1 NT x-L2hot", 16);
      variant(k_vcache<double, 2, 6, 4, 3, 12, 1, true>, "WL6 MAP1 NT no entries", 12);
      variant(k_vcache<double, 2, 4, 4, 3, 1>, "no x loads", 1);
      variant(k_vcache<double, 2, 4, 4, 3, 3>, "no x", 3);
      variant(k_vcache<double, 2, 4, 4, 3, 4>, "no entry loads", 4);
      variant(k_vcache<double, 2, 4, 4, 3, 8>, "no compute", 8);
      variant(k_vcache<double, 2, 4, 4, 3, 12>, "no entries/compute", 12);
      variant(k_vcache<double, 2, 4, 4, 3, 15>, "skeleton", 15);
      variant(k_vcache<double, 2, 4, 4, 3, 16>, "x L2-hot", 16);
      variant(k_vcache<double, 2, 4, 4, 3, 47>, "skeleton no barrier", 47);
    }
  }
  return 0;
}
