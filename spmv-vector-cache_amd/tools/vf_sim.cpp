// vf_sim: CPU replay of k_vflow's addressing and arithmetic (csrc/vflow.hip)
// over its layout (csrc/plan.cpp build_vflow), for checking on the host what
// the GPU would run.
//
// Per work unit (row block b, column part h) it replays the loader waves' DMA
// chunk placement into the LDS x slots (clamped source columns, the odd-cols
// patch) and every compute wave's steps: the group bounds it reads, the
// buffer-descriptor clamp (lanes past the group read code 0 and write nothing),
// the x / y LDS indices, the DPP first continuation (a run must stay inside a
// 16-lane row) and the shuffle tail, then the four-part combine in part order.
// Checked on every access: global indices inside their arrays, LDS indices
// inside the slot / y block, every y row updated only by the wave that owns it
// (vf_wave_of: the kernel's no-race premise across steps), every entry consumed
// exactly once.  The result is compared with a sequential CSR sum: u64 exact,
// f64 within the FAST bound.
//
// Test infrastructure (tests/test_vcache_sim.py); not part of the product.
#include <algorithm>
#include <cmath>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../host/Synthetic.h"
#include "hipspmv_internal.h"
#include "vc_map.h"

using namespace hipspmv;

static int g_errors = 0;
#define CHECK(cond, ...)                                                 \
  do {                                                                   \
    if (!(cond)) {                                                       \
      if (g_errors++ < 20) {                                             \
        std::fprintf(stderr, "VIOLATION %s:%d: ", __FILE__, __LINE__);   \
        std::fprintf(stderr, __VA_ARGS__);                               \
        std::fprintf(stderr, "\n");                                      \
      }                                                                  \
    }                                                                    \
  } while (0)

template <typename T>
static T mul(T a, T b) { return a * b; }

// one matrix: replay, compare; returns true when every check passed
template <typename T>
static bool replay(const char* name, const HostCSR& a, const std::vector<T>& x, int expect_eligible) {
  const int e0 = g_errors;
  VflowLayout V;
  const bool ok = build_vflow(a, V);
  if (expect_eligible >= 0 && ok != (expect_eligible == 1)) {
    std::printf("%s: eligibility %d, expected %d: FAIL\n", name, (int)ok, expect_eligible);
    return false;
  }
  if (!ok) {
    std::printf("%s: not eligible (as expected): ok\n", name);
    return true;
  }
  const VcacheLayout& L = V.L;
  const uint32_t S = kVfGeom.split, VP = kVfGeom.panel, WC = kVfWaves, WL = kVfLoaders, NS = kVfSlots;
  const uint32_t units = L.nblocks * S, npad = L.npad, cols = a.cols, rows = a.rows;
  CHECK(vcache_grid_ok(rows, cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels, npad, VP, S, kVfGeom),
        "grid");
  std::vector<int> used(a.nnz, 0);
  std::vector<std::vector<T>> part(S, std::vector<T>(rows, T(0)));
  const uint32_t cmax = (cols - 2) & ~1u;
  for (uint32_t slot = 0; slot < units; ++slot) {
    uint32_t b, h;
    vc_unit_map0<4>(slot, L.nblocks, b, h);
    const uint32_t r0 = b * L.rows_per_block, nr = std::min(L.rows_per_block, rows - r0);
    const uint32_t p0 = vc_part_first(h, L.npanels, S), npu = vc_part_first(h + 1, L.npanels, S) - p0;
    const uint32_t u = b * S + h;
    std::vector<T> y(kVfGeom.rows, T(0));
    std::vector<int> owner(kVfGeom.rows, -1);
    std::vector<T> xs(VP);
    for (uint32_t s = 0; s < npu; ++s) {
      // the DMA of loader wave s % WL (the whole panel): chunk j, lane pairs clamped to cmax
      std::vector<int> filled(VP, 0);
      CHECK(s % WL < WL, "loader");
      for (uint32_t j = 0; j < VP / 2 / 64; ++j)
          for (uint32_t lane = 0; lane < 64; ++lane) {
            const uint32_t c0 = j * 64, pr = c0 + lane;
            const uint32_t src = std::min((p0 + s) * VP + 2 * pr, cmax);
            CHECK(src + 1 < cols, "x pair %u past cols %u", src, cols);
            CHECK(2 * pr + 1 < VP, "slot index %u", 2 * pr);
            xs[2 * pr] = x[src];
            xs[2 * pr + 1] = x[src + 1];
            filled[2 * pr] = filled[2 * pr + 1] = 1;
          }
      if ((cols & 1) && p0 + s == L.npanels - 1) xs[cols - 1 - (p0 + s) * VP] = x[cols - 1];
      for (uint32_t i = 0; i < VP; ++i) CHECK(filled[i], "slot element %u never written", i);
      for (uint32_t cw = 0; cw < WC; ++cw) {
        const size_t gi = ((size_t)u * WC + cw) * npad + std::min(s, npad - 1);
        CHECK(gi < V.wbeg.size(), "wbeg index");
        const uint32_t e0 = V.wbeg[gi], n = V.wend[gi] - e0;
        CHECK(n <= kVfGroupMax, "group of %u entries", n);
        CHECK(e0 + n <= a.nnz, "group past nnz");
        // lanes of slots j = 0, 1: entry e0 + lane + 64 j when < n, else code 0
        uint32_t c[128];
        T v[128];
        for (uint32_t q = 0; q < 128; ++q) {
          c[q] = q < n ? L.code[e0 + q] : 0u;
          v[q] = q < n ? (T)__builtin_bit_cast(T, L.vals[e0 + q]) : T(0);
        }
        for (uint32_t q = 0; q < n; ++q) used[e0 + q]++;
        for (uint32_t q = 0; q < 128; ++q) {
          const uint32_t row = (c[q] >> 16) & 0x3FFF, col = c[q] & 0xFFFF;
          CHECK(col < VP, "x index %u", col);
          CHECK(row < (uint32_t)kVfGeom.rows, "y index %u", row);
          if (q >= n || (c[q] & kVcCont)) continue;
          CHECK(row < nr, "row %u past the block's %u", row, nr);
          CHECK(vf_wave_of(row) == cw, "row %u (wave %u) updated by wave %u", row, vf_wave_of(row), cw);
          CHECK(owner[row] < 0 || owner[row] == (int)cw, "row %u by two waves", row);
          owner[row] = (int)cw;
          CHECK((p0 + s) * VP + col < cols, "column past cols");
          T acc = y[row] + mul(v[q], xs[col]);
          uint32_t k = q;
          while (c[k] & kVcMore) {  // lane k + 1: DPP inside the 16-lane row, else and then shuffles
            ++k;
            CHECK(k < n && (c[k] & kVcCont), "run continues past its group");
            CHECK(k / 64 == q / 64, "run crosses a slot");
            if (k >= n) break;
            acc = acc + mul(v[k], xs[c[k] & 0xFFFF]);
          }
          y[row] = acc;
        }
      }
    }
    for (uint32_t r = 0; r < nr; ++r) part[h][r0 + r] = y[r];
  }
  for (uint32_t e = 0; e < a.nnz; ++e) CHECK(used[e] == 1, "entry %u consumed %d times", e, used[e]);
  // combine p0 + p1 + p2 + p3 (part order) vs the sequential CSR sums
  uint32_t bad = 0;
  double worst = 0;
  for (uint32_t r = 0; r < rows; ++r) {
    T yv = part[0][r];
    for (uint32_t q = 1; q < S; ++q) yv = yv + part[q][r];
    T ref = T(0);
    double absp = 0;
    for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e) {
      const T p = mul((T)__builtin_bit_cast(T, a.vals[e]), x[a.colind[e]]);
      ref = ref + p;
      if constexpr (std::is_floating_point_v<T>) absp += std::fabs((double)p);
    }
    if constexpr (std::is_floating_point_v<T>) {
      const double len = std::max<uint32_t>(1, a.rowptr[r + 1] - a.rowptr[r]);
      const double bound = 2.0 * len * std::ldexp(1.0, -53) * absp + 1e-300;
      const double err = std::fabs((double)yv - (double)ref);
      worst = std::max(worst, err / bound);
      if (err > bound) ++bad;
    } else if (yv != ref) {
      ++bad;
    }
  }
  CHECK(bad == 0, "%u rows outside the bound / not exact (worst err/bound %.3f)", bad, worst);
  const bool pass = g_errors == e0;
  std::printf("%s: %u units, %u steps, max group %u, worst err/bound %.3f: %s\n", name, units, L.part_panels,
              V.max_group, worst, pass ? "ok" : "FAIL");
  return pass;
}

static HostCSR stripe(uint32_t rows, uint32_t cols, uint32_t k, uint64_t seed) {
  HostCSR a;
  a.rows = rows;
  a.cols = cols;
  a.nnz = rows * k;
  a.rowptr.resize(rows + 1);
  a.colind.resize(a.nnz);
  a.vals.resize(a.nnz);
  std::vector<double> v(a.nnz);
  genStripeCSR(0, rows, cols, k, 1 + seed, 2 + seed, a.rowptr.data(), a.colind.data(), v.data());
  for (uint32_t e = 0; e < a.nnz; ++e) a.vals[e] = __builtin_bit_cast(uint64_t, v[e]);
  return a;
}

static HostCSR random_csr(uint32_t rows, uint32_t cols, uint32_t maxlen, uint64_t seed, bool clustered) {
  HostCSR a;
  a.rows = rows;
  a.cols = cols;
  a.rowptr.resize(rows + 1);
  std::vector<uint32_t> ci;
  std::vector<uint64_t> vv;
  uint64_t z = seed;
  auto rnd = [&] {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t q = z;
    q = (q ^ (q >> 30)) * 0xBF58476D1CE4E5B9ull;
    q = (q ^ (q >> 27)) * 0x94D049BB133111EBull;
    return q ^ (q >> 31);
  };
  a.rowptr[0] = 0;
  for (uint32_t r = 0; r < rows; ++r) {
    const uint32_t len = (uint32_t)(rnd() % (maxlen + 1));
    std::vector<uint32_t> cs;
    uint32_t c = (uint32_t)(rnd() % cols);
    for (uint32_t i = 0; i < len; ++i) {
      // clustered: runs of neighbouring columns (several entries of a row per panel)
      c = clustered ? (c + 1 + (uint32_t)(rnd() % 3)) % cols : (uint32_t)(rnd() % cols);
      cs.push_back(c);
    }
    std::sort(cs.begin(), cs.end());
    cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
    for (uint32_t cc : cs) {
      ci.push_back(cc);
      vv.push_back(__builtin_bit_cast(uint64_t, (double)((int64_t)(rnd() >> 12) - (1ll << 51)) * 0x1p-51));
    }
    a.rowptr[r + 1] = (uint32_t)ci.size();
  }
  a.nnz = (uint32_t)ci.size();
  a.colind.assign(ci.begin(), ci.end());
  a.vals.assign(vv.begin(), vv.end());
  return a;
}

int main(int argc, char** argv) {
  const bool full = argc > 1 && std::string(argv[1]) == "c3";
  bool all = true;
  auto xs = [](uint32_t n, uint64_t seed) {
    std::vector<double> x(n);
    for (uint32_t i = 0; i < n; ++i) x[i] = uniform11(splitmix64_at(seed, i));
    return x;
  };
  auto xu = [](uint32_t n) {
    std::vector<uint64_t> x(n);
    for (uint32_t i = 0; i < n; ++i) x[i] = (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    return x;
  };
  {
    HostCSR a = stripe(full ? 1u << 20 : 1u << 16, full ? 1u << 20 : 1u << 16, 32, 0);
    all &= replay<double>(full ? "stripe c3" : "stripe 2^16", a, xs(a.cols, 3), 1);
    all &= replay<uint64_t>(full ? "stripe c3 u64" : "stripe 2^16 u64", a, xu(a.cols), 1);
  }
  if (!full) {
    HostCSR b = stripe(70001, 40001, 8, 5);  // odd cols, partial row block, parts of 7-8 panels
    all &= replay<double>("stripe 70001x40001", b, xs(b.cols, 4), 1);
    all &= replay<uint64_t>("stripe 70001x40001 u64", b, xu(b.cols), 1);
    HostCSR c = random_csr(5000, 20001, 12, 7, true);  // runs of 2-12 inside a panel, some across DPP rows
    all &= replay<double>("clustered 5000x20001", c, xs(c.cols, 5), 1);
    all &= replay<uint64_t>("clustered 5000x20001 u64", c, xu(c.cols), 1);
    HostCSR d = random_csr(3000, 30001, 40, 9, false);  // ragged, empty rows
    all &= replay<double>("ragged 3000x30001", d, xs(d.cols, 6), 1);
    HostCSR e = random_csr(100, 3800, 8, 11, false);  // 3 panels, four parts: not eligible
    all &= replay<double>("narrow 100x3800", e, xs(e.cols, 7), 0);
  }
  std::printf(all && g_errors == 0 ? "vf_sim: all ok\n" : "vf_sim: FAILED\n");
  return all && g_errors == 0 ? 0 : 1;
}
