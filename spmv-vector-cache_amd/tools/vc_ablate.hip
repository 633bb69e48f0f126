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
#include <string>
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

template <typename V>
auto up(const V& v) {  // any contiguous host array (std::vector, the layouts' hvec)
  using T = std::remove_const_t<std::remove_reference_t<decltype(*v.data())>>;
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
  CK(hipMalloc(&dpart, 8ull * 4 * (n + 256 * 16384)));  // [split][nblocks][VRP] partials, split <= 4
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
  for (VcGeom g : {kVcOrdered, kVcSplit, kVcSplit4}) {
    VcacheLayout L;
    build_vcache(a, g, L);
    const bool dmawait = argc > 2 && std::string(argv[2]) == "dmawait";
    if (dmawait && g.split == 3) place_segments_banked(L, kVcSplitCT);  // the product layout (CX 5 needs it)
    // tickets: 2 per block for the combine + 8 stamp words per unit (AB & 128)
    uint32_t* dtick = up(std::vector<uint32_t>(2 * L.nblocks + 8 * L.nblocks * g.split, 0));
    VcacheArgs A{up(L.seg), up(L.code), up(L.vals), dx, dy, dy, dpart, dtick,
                 a.rows, a.cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels, L.npad, a.nnz - 1,
                 g.split, 0};
    std::printf("geometry rows=%d panel=%d split=%d: units=%u npad=%u max_seg=%u\n", g.rows, g.panel, g.split,
                L.nblocks * g.split, L.npad, L.max_seg);
    // kern must be compiled for this geometry (the round-1 fault was a split=1
    // kernel launched on the split layout's grid): SPLIT is checked here
    // window: entries a CX variant holds in registers per step (0: no limit)
    auto variant = [&](auto kern, int kernel_split, const char* nm, int mask, uint32_t window = 0) {
      if (kernel_split != g.split || !vcache_grid_ok(a.rows, a.cols, L.rows_per_block, L.nblocks, L.npanels,
                                                     L.part_panels, L.npad, (uint32_t)g.panel, g.split, g)) {
        std::printf("  %-30s SKIPPED: kernel split %d vs layout split %d\n", nm, kernel_split, g.split);
        return;
      }
      if (window && L.max_seg > window) {
        std::printf("  %-30s SKIPPED: max segment %u > register window %u\n", nm, L.max_seg, window);
        return;
      }
      const double us = timeit([&] {
        hipLaunchKernelGGL(kern, dim3(A.nblocks * A.split), dim3(kVcThreads), 0, nullptr, A.seg, A.code,
                           (const double*)A.vals, (const double*)A.x, (const double*)A.y_in, (double*)A.y_out,
                           (double*)A.partial, A.tickets, A.rows, A.cols, A.rows_per_block, A.nblocks, A.npanels,
                           A.part_panels, A.npad, A.last, A.beta, ~0u, (const uint64_t*)nullptr);
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
    // per-unit timeline of one launch (AB & 128: 8 stamp words per unit, csrc/vcache.hip)
    auto stamps = [&](auto kern, const char* nm) {
      const uint32_t units = A.nblocks * A.split;
      for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL(kern, dim3(units), dim3(kVcThreads), 0, nullptr, A.seg, A.code, (const double*)A.vals,
                           (const double*)A.x, (const double*)A.y_in, (double*)A.y_out, (double*)A.partial,
                           A.tickets, A.rows, A.cols, A.rows_per_block, A.nblocks, A.npanels, A.part_panels, A.npad,
                           A.last, A.beta, ~0u, (const uint64_t*)nullptr);
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> st(8 * units);
      const uint32_t* src = A.split == 1 ? reinterpret_cast<const uint32_t*>(A.partial) : A.tickets + 2 * A.nblocks;
      CK(hipMemcpy(st.data(), src, 4ull * st.size(), hipMemcpyDeviceToHost));
      uint32_t t0 = st[0];
      for (uint32_t u = 0; u < units; ++u)
        if ((int32_t)(st[8 * u] - t0) < 0) t0 = st[8 * u];
      auto us = [&](uint32_t u, int k) { return (int32_t)(st[8 * u + k] - t0) * 0.01; };
      std::vector<double> start, prolog, loop, tail_last, tail_pub, end, lwork, lwait, cwait;
      for (uint32_t u = 0; u < units; ++u) {
        start.push_back(us(u, 0));
        prolog.push_back(us(u, 1) - us(u, 0));
        loop.push_back(us(u, 2) - us(u, 1));
        end.push_back(us(u, 3));
        (A.split == 1 || st[8 * u + 4] == (uint32_t)A.split - 1 ? tail_last : tail_pub).push_back(us(u, 3) - us(u, 2));
        lwork.push_back(st[8 * u + 5] / 2400.0);  // s_memtime cycles at a nominal 2.4 GHz
        lwait.push_back(st[8 * u + 6] / 2400.0);
        cwait.push_back(st[8 * u + 7] / 2400.0);
      }
      auto q = [](std::vector<double> v, const char* what) {
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        std::printf("    %-26s min %7.2f  p10 %7.2f  median %7.2f  p90 %7.2f  max %7.2f us\n", what, v[0],
                    v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
      };
      std::printf("  stamps: %s (%u units; us from the first start)\n", nm, units);
      q(start, "start");
      q(prolog, "prologue");
      q(loop, "main loop");
      q(tail_pub, "publish (non-last)");
      q(tail_last, "combine / write (last)");
      q(end, "exit");
      q(lwork, "loader work (2.4 GHz)");
      q(lwait, "loader barrier wait");
      q(cwait, "compute barrier wait");
      for (uint32_t x = 0; x < 8; ++x) {  // by dispatch slot mod 8 (one XCD under round-robin placement)
        std::vector<double> lx;
        for (uint32_t u = x; u < units; u += 8) lx.push_back(loop[u]);
        std::sort(lx.begin(), lx.end());
        std::printf("    slot%%8=%u main loop median %7.2f max %7.2f\n", x, lx[lx.size() / 2], lx.back());
      }
    };
    if (dmawait) {  // round 6: the product against loaders that skip their DMA wait (AB 32768)
      if (g.split == 3)
        for (int r = 0; r < 4; ++r) {
          variant(k_vcache<double, 3, 3, 4, 2, 256, 0, false, 1, 5>, 3, "product (CX5, nt b >= nb/2)", 0,
                  13 * 64 * 2);
          variant(k_vcache<double, 3, 3, 4, 2, 256 | 32768, 0, false, 1, 5>, 3, "loaders skip the DMA wait", 32768,
                  13 * 64 * 2);
        }
      continue;
    }
    if (argc > 2 && std::string(argv[2]) == "stamps") {
      if (g.split == 3) {
        stamps(k_vcache<double, 3, 3, 4, 2, 128, 0, false, 1, 3>, "product (split 3)");
      } else if (g.split == 1) {
        stamps(k_vcache<double, 1, 8, 4, 3, 128>, "ordered vcache");
      }
      continue;
    }
    // template: <T, SPLIT, WL, DE, EPT, AB, MAP, NT, LD, CX>
    if (g.split == 1) {
      variant(k_vcache<double, 1>, 1, "default (WL8 DE4 EPT3)", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 0, 0, false, 0, 1>, 1, "xlane1", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 4, 3, 0, 0, false, 2, 2>, 1, "xlane2 (asm rings)", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 4, 3, 0, 0, false, 0, 3>, 1, "xlane3 (padded, compiler waits)", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 6, 3, 0, 0, false, 2, 2>, 1, "xlane2 DE6", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 4, 4, 2, 0, 0, false, 2, 2>, 1, "xlane2 WL4 EPT2", 0, 12 * 64 * 2);
      variant(k_vcache<double, 1, 8, 4, 3, 12, 0, false, 2, 2>, 1, "xlane2 no entries/compute", 12, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 4, 3, 3, 0, false, 2, 2>, 1, "xlane2 no x", 3, 8 * 64 * 3);
      variant(k_vcache<double, 1, 2, 4, 3, 0, 0, false, 1>, 1, "DMA WL2 DE4 EPT3", 0);
      variant(k_vcache<double, 1, 1, 4, 3, 0, 0, false, 1>, 1, "DMA WL1 DE4 EPT3", 0);
      variant(k_vcache<double, 1, 2, 4, 2, 0, 0, false, 1>, 1, "DMA WL2 DE4 EPT2", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 256>, 1, "default, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 1024>, 1, "default, nt b >= 3nb/8", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 2048>, 1, "default, nt b >= nb/4", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 512>, 1, "default, nt b >= 5nb/8", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 0, 0, true>, 1, "default, all nt", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 256, 0, false, 0, 3>, 1, "xlane3, nt b >= nb/2", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 4, 3, 1024, 0, false, 0, 3>, 1, "xlane3, nt b >= 3nb/8", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 6, 3, 256, 0, false, 2, 2>, 1, "xlane2 DE6, nt b >= nb/2", 0, 8 * 64 * 3);
      variant(k_vcache<double, 1, 8, 4, 3, 0, 0, true, 0, 3>, 1, "xlane3, all nt", 0, 8 * 64 * 3);
      // round 3: loader / compute balance with half the entries nt
      variant(k_vcache<double, 1, 6, 4, 3, 256>, 1, "WL6, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 10, 4, 3, 256>, 1, "WL10, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 4, 4, 3, 256, 0, false, 1>, 1, "DMA WL4, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 6, 4, 3, 256, 0, false, 1>, 1, "DMA WL6, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 8, 6, 3, 256>, 1, "DE6, nt b >= nb/2", 0);
      variant(k_vcache<double, 1, 8, 4, 3, 256 | 12>, 1, "nt b >= nb/2, x only", 12);
      variant(k_vcache<double, 1, 8, 4, 3, 256 | 3>, 1, "nt b >= nb/2, no x", 3);
      variant(k_vcache<double, 1, 8, 4, 3, 3>, 1, "no x", 3);
      variant(k_vcache<double, 1, 8, 4, 3, 12>, 1, "no entries/compute", 12);
      variant(k_vcache<double, 1, 8, 4, 3, 15>, 1, "skeleton", 15);
    } else if (g.split == 3) {  // the product FAST geometry (round 2)
      variant(k_vcache<double, 3, 3, 4, 2, 0, 0, false, 1, 3>, 3, "product (DMA WL3 DE4 EPT2, xlane3)", 0,
              13 * 64 * 2);
      // Infinity-Cache residency: the entries of the row blocks past a threshold non-temporal
      variant(k_vcache<double, 3, 3, 4, 2, 256, 0, false, 1, 3>, 3, "product, nt b >= nb/2", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 512, 0, false, 1, 3>, 3, "product, nt b >= 5nb/8", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 1024, 0, false, 1, 3>, 3, "product, nt b >= 3nb/8", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 0, 0, true, 1, 3>, 3, "product, all entries nt", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 2048, 0, false, 1, 3>, 3, "product, nt b >= nb/4", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 4096, 0, false, 1, 3>, 3, "product, nt b >= nb/8", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 0, 0, true, 1, 3>, 3, "product, all entries nt (again)", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 64, 0, true, 1, 3>, 3, "all nt, without the combine", 64, 13 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 0, 0, true, 1, 3>, 3, "all nt, DMA WL2", 0, 14 * 64 * 2);
      variant(k_vcache<double, 3, 4, 4, 2, 0, 0, true, 1, 3>, 3, "all nt, DMA WL4", 0, 12 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 0, 0, false, 1, 3>, 3, "product (again)", 0, 13 * 64 * 2);
      variant(k_vcache<double, 3, 3, 4, 2, 64, 0, false, 1, 3>, 3, "product without the combine", 64,
              13 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 0, 0, false, 1, 3>, 3, "DMA WL2 DE4 EPT2, xlane3", 0, 14 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 0, 0, false, 1, 0>, 3, "DMA WL2, runs re-read", 0);
      variant(k_vcache<double, 3, 4, 4, 3, 0, 0, false, 1, 3>, 3, "DMA WL4 EPT3 xlane3", 0, 12 * 64 * 3);
      variant(k_vcache<double, 3, 6, 4, 3, 0, 0, false, 0, 3>, 3, "registers WL6 EPT3 xlane3", 0, 10 * 64 * 3);
      variant(k_vcache<double, 3, 2, 4, 2, 3, 0, false, 1, 3>, 3, "no x", 3, 14 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 12, 0, false, 1, 3>, 3, "no entries/compute", 12, 14 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 15, 0, false, 1, 3>, 3, "skeleton", 15, 14 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 47, 0, false, 1, 3>, 3, "skeleton without step barriers", 47,
              14 * 64 * 2);
      variant(k_vcache<double, 3, 2, 4, 2, 111, 0, false, 1, 3>, 3, "... and without the combine", 111,
              14 * 64 * 2);
    } else {
      variant(k_vcache<double, 4>, 4, "default (WL2 DE4 EPT2)", 0);
      variant(k_vcache<double, 4, 2, 4, 2, 0, 0, false, 2, 2>, 4, "xlane2 (asm rings)", 0, 14 * 64 * 2);
      variant(k_vcache<double, 4, 2, 6, 2, 0, 0, false, 2, 2>, 4, "xlane2 DE6", 0, 14 * 64 * 2);
      variant(k_vcache<double, 4, 1, 4, 2, 0, 0, false, 1, 2>, 4, "xlane2 DMA WL1", 0, 15 * 64 * 2);
      variant(k_vcache<double, 4, 4, 4, 2>, 4, "WL4 DE4 EPT2", 0);
      variant(k_vcache<double, 4, 2, 6, 2>, 4, "WL2 DE6 EPT2", 0);
      variant(k_vcache<double, 4, 2, 4, 3>, 4, "WL2 DE4 EPT3", 0);
      variant(k_vcache<double, 4, 1, 4, 2, 0, 0, false, 1>, 4, "DMA WL1 DE4 EPT2", 0);
      variant(k_vcache<double, 4, 2, 4, 2, 0, 0, false, 1>, 4, "DMA WL2 DE4 EPT2", 0);
      variant(k_vcache<double, 4, 2, 4, 2, 3>, 4, "no x", 3);
      variant(k_vcache<double, 4, 2, 4, 2, 12>, 4, "no entries/compute", 12);
      variant(k_vcache<double, 4, 2, 4, 2, 15>, 4, "skeleton", 15);
    }
  }
  return 0;
}
