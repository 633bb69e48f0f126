// step_trace: where does a step of the C3 FAST kernel spend its time?
// (diagnostic, not part of the product libraries.)
//
// Builds the C3 matrix and the product's three-part layout, warms the chip up
// with 400 launches of the product kernel (past the DVFS transient of
// DESIGN.md §7), times it, then launches the same kernel with the step trace
// compiled in (k_vcache AB 8192 | 64: no combine) and reads, for every
// workgroup, wave and step, when the wave's data had landed (entries for a
// compute wave, the next x panel for a loader wave), when it reached the step
// barrier and when the barrier let it go (s_memtime, shader cycles).  Per step:
// the barrier releases when the last wave arrives; the summary says which
// role arrives last, how long the last arriver waited for memory and how long
// it then worked (LDS apply) before arriving.
//
//   make -C spmv-vector-cache_amd lib/step_trace && ./spmv-vector-cache_amd/lib/step_trace
#include "../csrc/vcache.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../host/Synthetic.h"

using namespace hipspmv;

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

template <typename T>
T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, sizeof(T) * std::max<size_t>(v.size(), 1)));
  CK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

struct Q {
  std::vector<double> v;
  void add(double x) { v.push_back(x); }
  void print(const char* what) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    std::printf("  %-44s mean %8.1f  p10 %8.1f  median %8.1f  p90 %8.1f  (cycles, n=%zu)\n", what, s / v.size(),
                v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.size());
  }
};

int main(int argc, char** argv) {
  const uint32_t n = 1u << 20, k = 32;
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
  // "ordered": the ORDERED geometry (SPLIT 1, 8 register-staged loader waves, its x-line mask)
  const bool ordered = argc > 1 && std::string(argv[1]) == "ordered";
  const VcGeom g = ordered ? kVcOrdered : kVcSplit;
  VcacheLayout L;
  build_vcache(a, g, L);
  const bool row_order = argc > 1 && std::string(argv[1]) == "roworder";
  if (!row_order) place_segments_banked(L, ordered ? kVcOrderedCT : kVcSplitCT);  // the product layouts (upload_vc)
  std::vector<uint64_t> xm;
  if (ordered) build_xmask(L, kVcOrderedLoaders, xm);
  const uint32_t units = L.nblocks * g.split;
  if (!vcache_grid_ok(a.rows, a.cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels, L.npad,
                      (uint32_t)g.panel, g.split, g) ||
      L.npad + 1 > 255 || L.max_seg > (ordered ? 8u * 64 * 3 : 13u * 64 * 2)) {
    std::printf("geometry check failed\n");
    return 1;
  }
  double* dx = up(x);
  double* dy;
  CK(hipMalloc(&dy, 8ull * n));
  // partials of the combine, and the trace (16 B per wave and step slot) in the same buffer
  const size_t part_bytes = std::max<size_t>(8ull * g.split * L.nblocks * ((L.rows_per_block + 1) & ~1u),
                                             16ull * units * 16 * 256);
  double* dpart;
  CK(hipMalloc(&dpart, part_bytes));
  uint32_t* dtick = up(std::vector<uint32_t>(4 * L.nblocks + 8 * units, 0));
  const uint32_t* dseg = up(L.seg);
  const uint64_t* dxm = ordered ? up(xm) : nullptr;
  const uint32_t* dcode = up(std::vector<uint32_t>(L.code.begin(), L.code.end()));
  const double* dvals = reinterpret_cast<const double*>(up(std::vector<uint64_t>(L.vals.begin(), L.vals.end())));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(units), dim3(kVcThreads), 0, nullptr, dseg, dcode, dvals, dx, (const double*)dy,
                       dy, dpart, dtick, a.rows, a.cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels,
                       L.npad, a.nnz - 1, 0, 0u, dxm);
  };
  // the product: xlane 5 on the banked layout (runs inside 16-lane rows), xlane 3 on the row-order one
  const bool x5 = !row_order && L.row_runs;
  auto product = ordered ? k_vcache<double, 1, 8, 4, 3, 0, 0, false, 0, 0>
                 : x5    ? k_vcache<double, 3, 3, 4, 2, 0, 0, false, 1, 5>
                         : k_vcache<double, 3, 3, 4, 2, 0, 0, false, 1, 3>;
  auto traced = ordered ? k_vcache<double, 1, 8, 4, 3, 8192 | 64, 0, false, 0, 0>
                : x5    ? k_vcache<double, 3, 3, 4, 2, 8192 | 64, 0, false, 1, 5>
                        : k_vcache<double, 3, 3, 4, 2, 8192 | 64, 0, false, 1, 3>;
  auto nocomb = ordered ? product
                : x5    ? k_vcache<double, 3, 3, 4, 2, 64, 0, false, 1, 5>
                        : k_vcache<double, 3, 3, 4, 2, 64, 0, false, 1, 3>;
  // configurations on the same layout (the register window must hold every segment)
  struct V {
    const char* name;
    void (*k)(const uint32_t*, const uint32_t*, const double*, const double*, const double*, double*, double*,
              uint32_t*, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, int,
              uint32_t, const uint64_t*);
    uint32_t window;
  };
  const V vars[] = {{"product", product, 13 * 64 * 2},
                    {"xlane 3 (WL3 DE4 EPT2)", k_vcache<double, 3, 3, 4, 2, 0, 0, false, 1, 3>, 13 * 64 * 2},
                    {"xlane 5 WL3 DE6", k_vcache<double, 3, 3, 6, 2, 0, 0, false, 1, 5>, 13 * 64 * 2},
                    {"xlane 5 WL2 DE4", k_vcache<double, 3, 2, 4, 2, 0, 0, false, 1, 5>, 14 * 64 * 2},
                    {"y by LDS atomic", k_vcache<double, 3, 3, 4, 2, 16384, 0, false, 1, 3>, 13 * 64 * 2},
                    {"WL2 DE4 EPT2", k_vcache<double, 3, 2, 4, 2, 0, 0, false, 1, 3>, 14 * 64 * 2},
                    {"WL2 DE4 EPT2 y atomic", k_vcache<double, 3, 2, 4, 2, 16384, 0, false, 1, 3>, 14 * 64 * 2},
                    {"WL3 DE6 EPT2", k_vcache<double, 3, 3, 6, 2, 0, 0, false, 1, 3>, 13 * 64 * 2},
                    {"WL3 DE3 EPT2", k_vcache<double, 3, 3, 3, 2, 0, 0, false, 1, 3>, 13 * 64 * 2},
                    {"WL4 DE4 EPT2", k_vcache<double, 3, 4, 4, 2, 0, 0, false, 1, 3>, 12 * 64 * 2}};
  auto timeit = [&](auto kern, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch(kern);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  for (int i = 0; i < 400; ++i) launch(product);
  CK(hipDeviceSynchronize());
  std::vector<double> y0(n), y1(n);
  launch(product);
  CK(hipMemcpy(y0.data(), dy, 8ull * n, hipMemcpyDeviceToHost));
  for (int round = 0; round < (ordered ? 0 : 3); ++round)
    for (const V& v : vars) {
      if (L.max_seg > v.window) continue;
      const double us = timeit(v.k, 100);
      launch(v.k);
      CK(hipMemcpy(y1.data(), dy, 8ull * n, hipMemcpyDeviceToHost));
      double md = 0;
      for (uint32_t i = 0; i < n; ++i) md = std::max(md, std::fabs(y1[i] - y0[i]) / (std::fabs(y0[i]) + 1e-300));
      std::printf("round %d  %-26s %8.2f us  max rel diff vs product %.1e\n", round, v.name, us, md);
    }
  std::printf("C3 %s, %u units, %u steps per unit: product %.2f us, without combine %.2f us, traced %.2f us\n",
              ordered ? "ORDERED" : "FAST", units, L.part_panels, timeit(product, 100), timeit(nocomb, 100),
              timeit(traced, 100));
  CK(hipMemset(dpart, 0, 16ull * units * 16 * 256));
  for (int i = 0; i < 20; ++i) launch(traced);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> tr(4ull * units * 16 * 256);
  CK(hipMemcpy(tr.data(), dpart, 4ull * tr.size(), hipMemcpyDeviceToHost));
  auto at = [&](uint32_t u, uint32_t w, uint32_t s, int f) { return tr[(((size_t)u * 16 + w) * 256 + s) * 4 + f]; };
  const uint32_t WL = ordered ? 8 : 3;
  Q step, crit_mem, crit_apply, crit_issue, crit_loader_mem, slack, comp_mem, comp_apply, comp_issue, loader_mem,
      prologue, spread;
  uint64_t crit_load = 0, crit_comp = 0;
  for (uint32_t u = 0; u < units; ++u) {
    const uint32_t h = ordered ? 0 : (u % (8 * 3)) / std::min(8u, L.nblocks - u / 24 * 8);
    const uint32_t npu = ordered ? L.npanels : vc_part_first(h + 1, L.npanels, 3) - vc_part_first(h, L.npanels, 3);
    uint32_t r_prev = UINT32_MAX, ent = UINT32_MAX;
    for (uint32_t w = 0; w < 16; ++w) {
      r_prev = std::min(r_prev, at(u, w, 255, 2));
      ent = std::min(ent, at(u, w, 255, 0));
    }
    prologue.add((int32_t)(r_prev - ent));
    for (uint32_t s = 0; s < npu; ++s) {
      uint32_t rel = UINT32_MAX, rel_max = 0, arr = 0, cw = 0;
      for (uint32_t w = 0; w < 16; ++w) {
        const uint32_t r = at(u, w, s, 2), ar = at(u, w, s, 1);
        rel = std::min(rel, r);
        rel_max = std::max(rel_max, r);
        if (w == 0 || (int32_t)(ar - r_prev) >= (int32_t)(arr - r_prev)) {
          arr = ar;
          cw = w;
        }
      }
      step.add((int32_t)(rel - r_prev));
      spread.add((int32_t)(rel_max - rel));
      slack.add((int32_t)(rel - arr));
      const double m = (int32_t)(at(u, cw, s, 0) - r_prev);
      if (cw < WL) {
        ++crit_load;
        crit_loader_mem.add(m);
      } else {
        ++crit_comp;
        crit_mem.add(m);
        crit_apply.add((int32_t)(at(u, cw, s, 3) - at(u, cw, s, 0)));
        crit_issue.add((int32_t)(arr - at(u, cw, s, 3)));
      }
      for (uint32_t w = 0; w < 16; ++w) {
        const double mw = (int32_t)(at(u, w, s, 0) - r_prev);
        if (w < WL) {
          loader_mem.add(mw);
        } else {
          comp_mem.add(mw);
          comp_apply.add((int32_t)(at(u, w, s, 3) - at(u, w, s, 0)));
          comp_issue.add((int32_t)(at(u, w, s, 1) - at(u, w, s, 3)));
        }
      }
      r_prev = rel;
    }
  }
  std::printf("steps traced: %llu; the last wave to arrive was a loader wave in %.1f %%, a compute wave in %.1f %%\n",
              (unsigned long long)(crit_load + crit_comp), 100.0 * crit_load / (crit_load + crit_comp),
              100.0 * crit_comp / (crit_load + crit_comp));
  prologue.print("prologue (entry -> first release)");
  step.print("step (release -> release)");
  crit_mem.print("last arriver, compute: memory wait");
  crit_apply.print("last arriver, compute: apply (LDS retired)");
  crit_issue.print("last arriver, compute: issue next loads");
  crit_loader_mem.print("last arriver, loader: panel landed");
  slack.print("last arrival -> release");
  spread.print("release spread over the waves");
  comp_mem.print("every compute wave: memory wait");
  comp_apply.print("every compute wave: apply (LDS retired)");
  comp_issue.print("every compute wave: issue next loads");
  loader_mem.print("every loader wave: panel landed");
  return 0;
}
