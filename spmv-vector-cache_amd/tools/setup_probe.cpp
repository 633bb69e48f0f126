// setup_probe: host-side phases of hipspmv_create_csr on a BASELINE matrix,
// timed on the CPU (no HIP: the device uploads are not in it) -- where the
// create time of full C4 goes.
//
//   setup_probe c4|c3|c5 [threads]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../host/Synthetic.h"
#include "hipspmv_internal.h"

using namespace hipspmv;

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "c4";
  std::vector<uint32_t> rowptr, colind;
  std::vector<double> vals;
  uint32_t n = 0;
  double t = now_s();
  if (which == "c5") {
    n = 1u << 24;
    genRmatCSR(24, 16, 4, 0.57, 0.19, 0.19, rowptr, colind, vals);
  } else {
    n = which == "c3" ? 1u << 20 : 1u << 24;
    const uint64_t nnz = (uint64_t)n * 32;
    rowptr.resize(n + 1);
    colind.resize(nnz);
    vals.resize(nnz);
    genStripeCSR(0, n, n, 32, 1, 2, rowptr.data(), colind.data(), vals.data());
  }
  const uint32_t nnz = rowptr[n];
  std::printf("%s: %u rows, %u nnz, generated in %.2f s\n", which.c_str(), n, nnz, now_s() - t);
  auto phase = [](const char* name, double t0) { std::printf("  %-34s %7.3f s\n", name, now_s() - t0); };
  HostCSR a;
  std::string why;
  t = now_s();
  copy_csr(rowptr.data(), colind.data(), vals.data(), n, n, nnz, a, why);
  phase("copy_csr", t);
  t = now_s();
  uint32_t maxlen = 0;
  for (uint32_t r = 0; r < a.rows; ++r) maxlen = std::max(maxlen, a.rowptr[r + 1] - a.rowptr[r]);
  phase("row lengths", t);
  t = now_s();
  std::vector<uint32_t> groups;
  build_row_groups(a, groups);
  phase("build_row_groups", t);
  const VcGeom geoms[] = {kVcOrdered, kVcSplit, kVcQuad, kWgWindow};
  const char* gname[] = {"vcache_eligible ordered", "vcache_eligible split", "vcache_eligible quad",
                         "vcache_eligible wgather"};
  bool wg = false;
  for (int i = 0; i < 4; ++i) {
    t = now_s();
    const bool e = vcache_eligible(a, geoms[i]);
    if (i == 3) wg = e;
    phase(gname[i], t);
  }
  if (wg) {
    t = now_s();
    (void)vcache_max_run(a, (uint32_t)kWgWindow.panel);
    phase("vcache_max_run wgather", t);
  }
  t = now_s();
  const uint64_t segs = windowed_segments(a, kWcLog2Window);
  phase("windowed_segments", t);
  std::printf("  (segments %llu)\n", (unsigned long long)segs);
  t = now_s();
  SellLayout S;
  build_sell(a, S);
  phase("build_sell", t);
  if (wg) {
    t = now_s();
    VcacheLayout W;
    build_vcache(a, kWgWindow, W);
    phase("build_vcache wgather", t);
    t = now_s();
    sort_segments_by_line(W);
    phase("sort_segments_by_line", t);
    t = now_s();
    VcacheLayout W2;
    build_vcache(a, kWgWindow, W2, true);
    phase("build_vcache wgather by line", t);
  }
  if (which == "c3") {  // the split layout and its LDS-bank placement (plan.cpp place_segments_banked)
    t = now_s();
    VcacheLayout V;
    build_vcache(a, kVcSplit, V);
    phase("build_vcache split", t);
    // LDS cycles per 32-lane half of the apply's ds_read_b64 (x: distinct columns by
    // column mod 32, y: rows by row mod 32) and per 16-lane quarter of its
    // ds_write_b64 (row mod 16), positions as k_vcache's compute lanes take them
    auto cost = [&](const VcacheLayout& L, double* out) {
      double cx = 0, cy = 0, cw = 0, groups = 0, quarters = 0;
      const uint32_t units = L.nblocks * 3, CT = kVcSplitCT;
      for (uint32_t u = 0; u < units; ++u)
        for (uint32_t i = 0; i < L.npad; ++i) {
          const uint32_t s0 = L.seg[(size_t)u * (L.npad + 1) + i], s1 = L.seg[(size_t)u * (L.npad + 1) + i + 1];
          if (s1 - s0 > 2 * CT) continue;
          for (uint32_t g0 = s0; g0 < s1; g0 += 32) {
            int mc[32] = {0}, my[32] = {0}, mw[2][16] = {{0}};
            std::vector<uint32_t> cols;
            for (uint32_t e = g0; e < std::min(s1, g0 + 32); ++e) {
              const uint32_t c = L.code[e] & 0xFFFF, r = (L.code[e] >> 16) & 0x3FFF;
              if (std::find(cols.begin(), cols.end(), c) == cols.end()) {
                cols.push_back(c);
                mc[c & 31]++;
              }
              if (!(L.code[e] & kVcCont)) {
                my[r & 31]++;
                mw[(e - g0) / 16][r & 15]++;
              }
            }
            cx += *std::max_element(mc, mc + 32);
            cy += std::max(1, *std::max_element(my, my + 32));
            for (int q = 0; q < 2; ++q) {
              cw += std::max(1, *std::max_element(mw[q], mw[q] + 16));
              quarters += 1;
            }
            groups += 1;
          }
        }
      out[0] = cx / groups;
      out[1] = cy / groups;
      out[2] = cw / quarters;
    };
    double c0[3], c1[3];
    cost(V, c0);
    t = now_s();
    place_segments_banked(V, kVcSplitCT);
    phase("place_segments_banked", t);
    cost(V, c1);
    std::printf("  LDS cycles per group (x read / y read / y write quarter): row order %.2f / %.2f / %.2f, "
                "banked %.2f / %.2f / %.2f\n", c0[0], c0[1], c0[2], c1[0], c1[1], c1[2]);
  }
  if (which == "c5") {
    t = now_s();
    WinLayout L;
    build_windowed(a, kWcLog2Window, L, (uint32_t)kCvGroupNnz);
    phase("build_windowed", t);
  }
  return 0;
}
