// CPU replay of k_sell (csrc/sell.hip) on the product layout (csrc/plan.cpp
// build_sell): every wave's loads at the indices the kernel forms (the
// software-pipelined pairs with their clamped prefetch, the hub stages with
// their clamped entries), bounds-checked; every row written exactly once; the
// arithmetic in the kernel's order -- ORDERED bit-exact against the CSR
// reference, FAST (hub rows: lane partials + xor tree, replayed lane by lane)
// within the FAST bound, u64 exact.  Test infrastructure (tests/test_sell_sim.py).
//
//   sell_sim [small]
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <type_traits>
#include <vector>

#include "hipspmv_internal.h"
#include "../host/Synthetic.h"

using namespace hipspmv;

static int g_violations = 0;
static void violation(const char* what, uint64_t i, uint64_t n) {
  if (g_violations++ < 10) std::fprintf(stderr, "VIOLATION %s: index %llu of %llu\n", what,
                                        (unsigned long long)i, (unsigned long long)n);
}
template <typename V>
static auto at(const V& v, uint64_t i, const char* what) -> decltype(v[0]) {
  if (i >= v.size()) {
    violation(what, i, v.size());
    return v[0];
  }
  return v[i];
}

template <typename T>
static T bits(uint64_t u) {
  T t;
  std::memcpy(&t, &u, 8);
  return t;
}

template <typename T>
static T neg_zero() {
  if constexpr (std::is_floating_point_v<T>)
    return -0.0;
  else
    return T(0);  // u64 never takes the chain (integer sums are order-free)
}

// The kernel's arithmetic for one element type.  mode: 0 FAST, 1 EXACT (hub chain).
template <typename T>
static std::vector<T> replay(const HostCSR& a, const SellLayout& L, const std::vector<T>& x,
                             const std::vector<T>& yin, int beta, bool exact, std::vector<int>& writes) {
  std::vector<T> y(a.rows, T(0));
  writes.assign(a.rows, 0);
  auto xv = [&](uint32_t c) { return at(x, c, "x gather"); };
  // the hub-entry routine (hub_entries): EXACT chain from acc, or lane
  // partials + xor tree; loads at the kernel's clamped indices
  auto hub_entries = [&](uint32_t base, uint32_t n, T acc, bool chain) -> T {
    if (chain) {  // hub_row_exact: stages of 64 * kChainG, lane l holds entries l*G .. l*G+G-1
      constexpr uint32_t G = kChainG, S = 64 * G;
      auto entry = [&](uint32_t g0, int lane, uint32_t j, uint32_t& c, T& v) {
        const uint32_t e = std::min<uint32_t>(g0 + (uint32_t)lane * G + j, n - 1);
        c = at(a.colind, (uint64_t)base + e, "hub colind");
        v = bits<T>(at(a.vals, (uint64_t)base + e, "hub vals"));
      };
      for (uint32_t g0 = 0; g0 < n; g0 += S) {
        for (int lane = 0; lane < 64; ++lane)
          for (uint32_t j = 0; j < G; ++j) {  // prefetches: entries two stages ahead, gathers one ahead
            uint32_t c;
            T v;
            entry(g0 + 2 * S, lane, j, c, v);
            entry(g0 + S, lane, j, c, v);
            (void)xv(c);
          }
        // the chain visits the lanes in order; an invalid product is -0.0
        for (int lane = 0; lane < 64; ++lane)
          for (uint32_t j = 0; j < G; ++j) {
            uint32_t c;
            T v;
            entry(g0, lane, j, c, v);
            const T p = g0 + (uint32_t)lane * G + j < n ? v * xv(c) : neg_zero<T>();
            acc = acc + p;
          }
      }
      return acc;
    }
    const uint32_t S = 256;
    auto entry = [&](uint32_t g0, int j, int lane, uint32_t& c, T& v) {
      const uint32_t e = std::min<uint32_t>(g0 + j * 64 + lane, n - 1);
      c = at(a.colind, (uint64_t)base + e, "hub colind");
      v = bits<T>(at(a.vals, (uint64_t)base + e, "hub vals"));
    };
    std::vector<std::array<T, 4>> part(64, {T(0), T(0), T(0), T(0)});
    for (uint32_t g0 = 0; g0 < n; g0 += S) {
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 4; ++j) {  // prefetches: entries two stages ahead, gathers one ahead
          uint32_t c;
          T v;
          entry(g0 + 2 * S, j, lane, c, v);
          entry(g0 + S, j, lane, c, v);
          (void)xv(c);
        }
      const uint32_t m = std::min(S, n - g0);
      if (chain) {
        for (uint32_t i = 0; i < m; ++i) {
          uint32_t c;
          T v;
          entry(g0, (int)(i >> 6), (int)(i & 63), c, v);
          const T p = v * xv(c);
          acc = acc + p;
        }
      } else {
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 4; ++j) {
            uint32_t c;
            T v;
            entry(g0, j, lane, c, v);
            const T p = v * xv(c);
            if (g0 + (uint32_t)(j * 64 + lane) < n) part[lane][j] = part[lane][j] + p;
          }
      }
    }
    if (chain) return acc;
    std::array<T, 64> s;
    for (int l = 0; l < 64; ++l) s[l] = (part[l][0] + part[l][1]) + (part[l][2] + part[l][3]);
    for (int d = 32; d >= 1; d >>= 1) {
      std::array<T, 64> t;
      for (int l = 0; l < 64; ++l) t[l] = s[l] + s[l ^ d];
      s = t;
    }
    for (int l = 1; l < 64; ++l)
      if (std::memcmp(&s[l], &s[0], 8)) violation("xor tree lanes disagree", l, 64);
    return s[0];
  };
  if (exact) {  // hub rows, one wave each
    for (uint32_t w = 0; w < L.nhubs; ++w) {
      const uint32_t r = at(L.hubs, w, "hubs");
      const uint32_t base = at(a.rowptr, r, "rowptr"), n = at(a.rowptr, (uint64_t)r + 1, "rowptr") - base;
      if (n <= kSellHub) violation("hub row too short", n, kSellHub);
      y[r] = hub_entries(base, n, beta ? yin[r] : T(0), true);
      writes[r]++;
    }
  } else {  // hub pieces; a row's pieces contiguous, combined in piece order
    std::vector<T> partial(L.npieces);
    std::vector<uint32_t> covered(a.rows, 0);
    for (uint32_t pid = 0; pid < L.npieces; ++pid) {
      const uint64_t w0 = (uint64_t)pid * kSellPieceWords;
      const uint32_t r = at(L.pieces, w0, "pieces"), begin = at(L.pieces, w0 + 1, "pieces"),
                     n = at(L.pieces, w0 + 2, "pieces"), idx = at(L.pieces, w0 + 3, "pieces"),
                     np = at(L.pieces, w0 + 4, "pieces"), tk = at(L.pieces, w0 + 5, "pieces");
      if (r >= a.rows || n == 0 || n > kSellPiece || idx >= np || pid < idx ||
          (np > 1 && tk >= L.ntickets)) {
        violation("piece record", pid, L.npieces);
        continue;
      }
      const uint32_t rb = a.rowptr[r], rn = a.rowptr[r + 1] - rb;
      if (begin != covered[r] || begin + n > rn) violation("piece range", begin, rn);
      covered[r] = begin + n;
      const T s = hub_entries(rb + begin, n, T(0), false);
      if (np == 1) {
        y[r] = beta ? yin[r] + s : s;
        writes[r]++;
        continue;
      }
      partial[pid] = s;
      if (idx == np - 1) {  // the combine reads every piece of the row in order, whoever arrives last
        T t = partial[pid - idx];
        for (uint32_t q = 1; q < np; ++q) t = t + partial[pid - idx + q];
        y[r] = beta ? yin[r] + t : t;
        writes[r]++;
      }
    }
    for (uint32_t r : L.hubs)
      if (covered[r] != a.rowptr[r + 1] - a.rowptr[r]) violation("hub row not covered by its pieces", r, a.rows);
  }
  // slice waves
  for (uint32_t s = 0; s < L.nslices; ++s) {
    const uint64_t off = at(L.off, s, "off"), end = at(L.off, (uint64_t)s + 1, "off");
    const uint32_t width = at(L.width, s, "width");
    if (end - off != (uint64_t)width * kSellRows) violation("slice size", end - off, (uint64_t)width * kSellRows);
    for (int lane = 0; lane < 64; ++lane) {
      uint32_t r[4], n[4];
      T acc[4];
      for (int j = 0; j < 4; ++j) {
        const uint64_t i = (uint64_t)s * kSellRows + j * 64 + lane;
        r[j] = at(L.row, i, "row");
        n[j] = at(L.len, i, "len");
        if (n[j] > width) violation("len > width", n[j], width);
        acc[j] = beta && r[j] != kSellNoRow ? at(yin, r[j], "y_in") : T(0);
      }
      // the index of step k, sub-slice j of this lane
      auto idx = [&](uint32_t k, int j) {
        const uint64_t i = off + ((uint64_t)k * 4 + j) * 64 + lane;
        if (i >= end) violation("slice entry outside its slice", i, end);
        return i;
      };
      auto step = [&](uint32_t k) {
        for (int j = 0; j < 4; ++j) {
          const uint64_t i = idx(k, j);
          const T t = acc[j] + bits<T>(at(L.vals, i, "sell vals")) * xv(at(L.col, i, "sell col"));
          if (k < n[j]) acc[j] = t;
        }
      };
      uint32_t k = 0;
      if (width >= 4) {
        for (int j = 0; j < 8; ++j) (void)idx(j >> 2, j & 3);  // load2(0)
        for (; k + 4 <= width; k += 4) {
          for (int q = 0; q < 8; ++q) (void)idx(k + 2 + (q >> 2), q & 3);  // load2(k + 2)
          const uint32_t kn = std::min(k + 4, width - 2);
          for (int q = 0; q < 8; ++q) (void)idx(kn + (q >> 2), q & 3);  // load2(clamped)
          step(k);
          step(k + 1);
          step(k + 2);
          step(k + 3);
        }
      }
      for (; k < width; ++k) step(k);
      for (int j = 0; j < 4; ++j)
        if (r[j] != kSellNoRow) {
          if (r[j] >= a.rows) {
            violation("row id", r[j], a.rows);
            continue;
          }
          y[r[j]] = acc[j];
          writes[r[j]]++;
        }
    }
  }
  return y;
}

template <typename T>
static std::vector<T> reference(const HostCSR& a, const std::vector<T>& x, const std::vector<T>& yin, int beta) {
  std::vector<T> y(a.rows);
  for (uint32_t r = 0; r < a.rows; ++r) {
    T acc = beta ? yin[r] : T(0);
    for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e) acc = acc + bits<T>(a.vals[e]) * x[a.colind[e]];
    y[r] = acc;
  }
  return y;
}

static HostCSR from_lens(const std::vector<uint32_t>& lens, uint32_t cols, uint64_t seed) {
  HostCSR A;
  A.rows = (uint32_t)lens.size();
  A.cols = cols;
  A.rowptr.assign(A.rows + 1, 0);
  std::mt19937_64 g(seed);
  for (uint32_t r = 0; r < A.rows; ++r) {
    const uint32_t n = std::min(lens[r], cols);
    std::vector<uint32_t> cs;
    if (n * 2 > cols) {
      for (uint32_t c = 0; c < cols; ++c) cs.push_back(c);
      std::shuffle(cs.begin(), cs.end(), g);
      cs.resize(n);
    } else {
      while (cs.size() < n) {
        const uint32_t c = (uint32_t)(g() % cols);
        bool dup = false;
        for (uint32_t d : cs) dup |= d == c;
        if (!dup) cs.push_back(c);
      }
    }
    std::sort(cs.begin(), cs.end());
    for (uint32_t c : cs) {
      A.colind.push_back(c);
      const double v = uniform11(g());
      uint64_t u;
      std::memcpy(&u, &v, 8);
      A.vals.push_back(u);
    }
    A.rowptr[r + 1] = (uint32_t)A.colind.size();
  }
  A.nnz = (uint32_t)A.colind.size();
  return A;
}

int main(int argc, char** argv) {
  const bool small = argc > 1 && std::string(argv[1]) == "small";
  struct Case {
    std::string name;
    HostCSR A;
  };
  std::vector<Case> cases;
  {  // C3-like stripe (uniform 32): no padding, no hubs
    const uint32_t n = small ? 1u << 12 : 1u << 16, k = 32;
    HostCSR A;
    A.rows = A.cols = n;
    A.nnz = n * k;
    A.rowptr.resize(n + 1);
    A.colind.resize(A.nnz);
    std::vector<double> v(A.nnz);
    genStripeCSR(0, n, n, k, 1, 2, A.rowptr.data(), A.colind.data(), v.data());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"stripe " + std::to_string(n), std::move(A)});
  }
  {  // R-MAT: skewed, hub rows, empty rows
    std::vector<uint32_t> rp, ci;
    std::vector<double> v;
    const uint32_t sc = small ? 12 : 15;
    genRmatCSR(sc, 16, 4, 0.57, 0.19, 0.19, rp, ci, v);
    HostCSR A;
    A.rows = A.cols = 1u << sc;
    A.nnz = (uint32_t)ci.size();
    A.rowptr.assign(rp.begin(), rp.end());
    A.colind.assign(ci.begin(), ci.end());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"rmat s" + std::to_string(sc), std::move(A)});
  }
  {  // ragged: widths 0..9 (odd tails), a few hub rows of assorted lengths
    std::mt19937_64 g(7);
    std::vector<uint32_t> lens(3001);
    for (auto& l : lens) l = (uint32_t)(g() % 10);
    lens[5] = 257;    // just over the hub threshold: one stage + 1
    lens[77] = 513;   // two full stages + 1
    lens[1000] = 700; // partial last stage
    lens[3000] = 256; // at the threshold: stays in a slice
    cases.push_back({"ragged 3001x2000", from_lens(lens, 2000, 11)});
  }
  {  // more rows than one sorting window, a slice tail in every window
    std::mt19937_64 g(9);
    std::vector<uint32_t> lens(small ? 70001 : 140001);
    for (auto& l : lens) l = (uint32_t)(g() % 40 == 0 ? 100 + g() % 150 : g() % 6);
    cases.push_back({"windows " + std::to_string(lens.size()), from_lens(lens, 5003, 13)});
  }
  {  // all rows empty; one row; one column
    cases.push_back({"empty 1000", from_lens(std::vector<uint32_t>(1000, 0), 17, 1)});
    cases.push_back({"single row 1x4000 (hub)", from_lens(std::vector<uint32_t>(1, 3000), 4000, 2)});
    // hub rows in several FAST pieces (combine in piece order)
    std::vector<uint32_t> lens(700, 3);
    lens[0] = 20000;  // 5 pieces
    lens[333] = 4097; // 2 pieces, the smallest split
    lens[699] = 8192; // 2 full pieces
    cases.push_back({"split hubs 700x30000", from_lens(lens, 30000, 4)});
    cases.push_back({"single column 300x1", from_lens(std::vector<uint32_t>(300, 1), 1, 3)});
  }
  int failures = 0;
  for (auto& cs : cases) {
    const HostCSR& A = cs.A;
    SellLayout L;
    build_sell(A, L);
    std::vector<double> x(A.cols), yin(A.rows);
    for (uint32_t i = 0; i < A.cols; ++i) x[i] = uniform11(splitmix64_at(3, i));
    for (uint32_t i = 0; i < A.rows; ++i) yin[i] = uniform11(splitmix64_at(5, i));
    std::vector<uint64_t> xu(A.cols), yu(A.rows);
    for (uint32_t i = 0; i < A.cols; ++i) xu[i] = splitmix64_at(6, i);
    for (uint32_t i = 0; i < A.rows; ++i) yu[i] = splitmix64_at(7, i);
    for (int beta = 0; beta < 2; ++beta) {
      for (int mode = 0; mode < 3; ++mode) {  // 0: f64 ORDERED, 1: f64 FAST, 2: u64
        g_violations = 0;
        std::vector<int> writes;
        size_t bad = 0;
        if (mode < 2) {
          const auto y = replay<double>(A, L, x, yin, beta, mode == 0, writes);
          const auto r = reference<double>(A, x, yin, beta);
          for (uint32_t i = 0; i < A.rows; ++i) {
            if (mode == 0) {
              bad += std::memcmp(&y[i], &r[i], 8) != 0;
            } else {
              double absp = beta ? std::fabs(yin[i]) : 0.0;
              const uint32_t len = A.rowptr[i + 1] - A.rowptr[i];
              for (uint32_t e = A.rowptr[i]; e < A.rowptr[i + 1]; ++e)
                absp += std::fabs(bits<double>(A.vals[e]) * x[A.colind[e]]);
              bad += !(std::fabs(y[i] - r[i]) <= 2.0 * (len + 1) * 0x1.0p-53 * absp + 1e-300);
            }
          }
        } else {
          const auto y = replay<uint64_t>(A, L, xu, yu, beta, false, writes);
          const auto r = reference<uint64_t>(A, xu, yu, beta);
          for (uint32_t i = 0; i < A.rows; ++i) bad += y[i] != r[i];
        }
        size_t miswritten = 0;
        for (int w : writes) miswritten += w != 1;
        const bool ok = bad == 0 && miswritten == 0 && g_violations == 0;
        failures += !ok;
        std::printf("%-26s %s beta=%d slices=%u hubs=%u pieces=%u padding=%llu: %s (%zu rows off, %zu rows not written once, "
                    "%d violations)\n",
                    cs.name.c_str(), mode == 0 ? "f64-ordered" : mode == 1 ? "f64-fast" : "u64", beta, L.nslices,
                    L.nhubs, L.npieces, (unsigned long long)L.padding, ok ? "ok" : "FAIL", bad, miswritten, g_violations);
      }
    }
  }
  return failures ? 1 : 0;
}
