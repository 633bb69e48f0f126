// vq_sim: CPU replay of k_vquad (csrc/vquad.hip) over the build_vcache_lanes
// placement (csrc/plan.cpp), for checking the layout and the kernel's step
// semantics on the host before a GPU sees them.
//
// Every unit (b, h) is replayed step by step the way the compute lanes run it:
// lane ct reads positions ct and CT + ct of the step's segment (out-of-range
// positions read nothing), forms both products from the x panel, a run head
// adds its lane's second entry (kVqLMore) or the next lanes of its wave
// (kVcMore, never past the wave), and owners update their y row.  Checked: x
// indices inside the panel, y rows inside the block, at most one owner per row
// per step, no kVcMore run leaving its wave or slot row, every entry of every
// segment consumed exactly once; the combine p0 + p1 + p2 + p3; and the result
// -- u64 exactly equal to a sequential CSR sum, f64 within the FAST bound.
// Test infrastructure (tests/test_vcache_sim.py); not part of the product.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../host/Synthetic.h"
#include "hipspmv_internal.h"

using namespace hipspmv;

static int g_err = 0;
#define CHECK(c, ...)                                                     \
  do {                                                                    \
    if (!(c)) {                                                           \
      if (g_err++ < 20) {                                                 \
        std::fprintf(stderr, "VIOLATION %s:%d: ", __FILE__, __LINE__);    \
        std::fprintf(stderr, __VA_ARGS__);                                \
        std::fprintf(stderr, "\n");                                       \
      }                                                                   \
    }                                                                     \
  } while (0)

template <typename T>
static T mul(T a, T b) {
  return a * b;
}

// y = A x through the layout, as k_vquad computes it (T: double or uint64_t)
template <typename T>
static std::vector<T> replay(const HostCSR& A, const VcacheLayout& L, const std::vector<T>& x) {
  const uint32_t CT = kVqLanes, P = (uint32_t)kVcQuad.panel, S = 4, R = L.rows_per_block;
  std::vector<T> y(A.rows, T(0));
  std::vector<uint8_t> seen(A.nnz, 0);
  auto val = [&](uint32_t e) { return __builtin_bit_cast(T, L.vals[e]); };
  for (uint32_t b = 0; b < L.nblocks; ++b) {
    const uint32_t r0 = b * R, nr = std::min(R, A.rows - r0);
    std::vector<std::vector<T>> part(S, std::vector<T>(nr, T(0)));
    for (uint32_t h = 0; h < S; ++h) {
      const uint32_t p0 = vc_part_first(h, L.npanels, S), npu = vc_part_first(h + 1, L.npanels, S) - p0;
      const uint32_t* sg = &L.seg[((size_t)b * S + h) * (L.npad + 1)];
      std::vector<T>& yl = part[h];
      for (uint32_t s = 0; s < npu; ++s) {
        const uint32_t beg = sg[s], end = sg[s + 1], n = end - beg;
        CHECK(n <= 2 * CT, "segment of %u entries past the register window", n);
        const uint32_t c0 = (p0 + s) * P, pw = std::min(P, A.cols - c0);  // this panel's columns
        std::vector<uint8_t> owner(nr, 0);
        for (uint32_t ct = 0; ct < CT; ++ct) {
          T p[2] = {T(0), T(0)};
          uint32_t code[2] = {0, 0}, row[2] = {0, 0};
          bool own[2] = {false, false}, valid[2];
          for (int j = 0; j < 2; ++j) {
            const uint32_t q = ct + j * CT;
            valid[j] = q < n;
            if (!valid[j]) continue;
            code[j] = L.code[beg + q];
            const uint32_t col = code[j] & 0xFFF;
            CHECK(col < pw, "x index %u past the panel's %u columns", col, pw);
            p[j] = mul(val(beg + q), x[c0 + std::min(col, pw - 1)]);
            own[j] = !(code[j] & kVcCont);
            row[j] = (code[j] >> 12) & 0x3FFF;
            CHECK(row[j] < nr, "y row %u past the block's %u rows", row[j], nr);
            row[j] = std::min(row[j], nr - 1);
          }
          T acc[2];
          for (int j = 0; j < 2; ++j) {
            if (!own[j]) continue;
            CHECK(!owner[row[j]], "two owners of row %u in one step", row[j]);
            owner[row[j]] = 1;
            acc[j] = yl[row[j]] + p[j];
            seen[beg + ct + j * CT] ^= 1;
            if (j == 0 && (code[0] & kVqLMore)) {
              CHECK(valid[1] && (code[1] & kVcCont) && ((code[1] >> 12) & 0x3FFF) == row[0],
                    "kVqLMore without its pair at lane %u", ct);
              acc[0] = acc[0] + p[1];
              seen[beg + ct + CT] ^= 1;
            }
            // kVcMore: the next lanes of the same wave, same slot row
            uint32_t q = ct + j * CT, cd = code[j];
            while (cd & kVcMore) {
              ++q;
              CHECK((q % CT) / 64 == (ct / 64) && q / CT == (uint32_t)j && q < n,
                    "kVcMore run leaves its wave / slot row at position %u", q);
              if (q >= n) break;
              cd = L.code[beg + q];
              CHECK((cd & kVcCont) && ((cd >> 12) & 0x3FFF) == row[j], "broken run at position %u", q);
              acc[j] = acc[j] + mul(val(beg + q), x[c0 + std::min(cd & 0xFFF, pw - 1)]);
              seen[beg + q] ^= 1;
            }
            yl[row[j]] = acc[j];
          }
        }
      }
    }
    for (uint32_t i = 0; i < nr; ++i) {  // y = p0 + p1 + p2 + p3 in part order
      T a = part[0][i];
      for (uint32_t h = 1; h < S; ++h) a = a + part[h][i];
      y[r0 + i] = a;
    }
  }
  for (uint32_t e = 0; e < A.nnz; ++e) CHECK(seen[e] == 1, "entry %u consumed %u times", e, seen[e]);
  return y;
}

static HostCSR random_csr(uint32_t rows, uint32_t cols, uint32_t maxlen, uint64_t seed, int dup) {
  HostCSR a;
  a.rows = rows;
  a.cols = cols;
  a.rowptr.assign(rows + 1, 0);
  uint64_t z = seed;
  auto rnd = [&]() {
    z += 0x9E3779B97F4A7C15ull;
    uint64_t v = z;
    v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
    v = (v ^ (v >> 27)) * 0x94D049BB133111EBull;
    return v ^ (v >> 31);
  };
  for (uint32_t r = 0; r < rows; ++r) {
    uint32_t len = (uint32_t)(rnd() % (maxlen + 1));
    if (r % 97 == 5) len = std::min<uint32_t>(cols, 100);  // rows with many entries per panel (long runs)
    std::vector<uint32_t> cs;
    for (uint32_t k = 0; k < len; ++k) cs.push_back((uint32_t)(rnd() % cols));
    std::sort(cs.begin(), cs.end());
    if (dup)
      for (size_t k = 0; k + 1 < cs.size(); k += 7) cs[k + 1] = cs[k];  // repeated columns
    for (uint32_t c : cs) {
      a.colind.push_back(c);
      a.vals.push_back(rnd());
    }
    a.rowptr[r + 1] = (uint32_t)a.colind.size();
  }
  a.nnz = (uint32_t)a.colind.size();
  return a;
}

template <typename T>
static void check_case(const char* name, const HostCSR& A, bool f64) {
  VcacheLayout L;
  if (!vcache_eligible(A, kVcQuad)) {
    std::printf("%-28s not eligible\n", name);
    return;
  }
  if (!build_vcache_lanes(A, kVcQuad, kVqLanes, L)) {
    std::printf("%-28s lanes placement refused (segment past the window or an unplaceable run)\n", name);
    return;
  }
  HostCSR B = A;
  std::vector<T> x(A.cols);
  for (uint32_t i = 0; i < A.cols; ++i) {
    const uint64_t z = splitmix64_at(9, i);
    x[i] = f64 ? __builtin_bit_cast(T, uniform11(z)) : __builtin_bit_cast(T, z);
  }
  if (f64)
    for (auto& v : B.vals) v = __builtin_bit_cast(uint64_t, uniform11(v));
  VcacheLayout Lf;
  build_vcache_lanes(B, kVcQuad, kVqLanes, Lf);
  const int before = g_err;
  const std::vector<T> y = replay<T>(B, Lf, x);
  uint32_t bad = 0;
  for (uint32_t r = 0; r < A.rows; ++r) {
    T ref = T(0);
    double absum = 0;
    for (uint32_t e = B.rowptr[r]; e < B.rowptr[r + 1]; ++e) {
      const T v = __builtin_bit_cast(T, B.vals[e]);
      ref = ref + mul(v, x[B.colind[e]]);
      if (f64) absum += std::fabs((double)v * (double)x[B.colind[e]]);
    }
    if (f64) {
      const double len = B.rowptr[r + 1] - B.rowptr[r];
      const double bound = 2.0 * std::max(len, 1.0) * std::ldexp(1.0, -53) * absum + 1e-300;
      if (std::fabs((double)y[r] - (double)ref) > bound) ++bad;
    } else if (std::memcmp(&y[r], &ref, sizeof(T))) {
      ++bad;
    }
  }
  CHECK(bad == 0, "%s: %u rows wrong", name, bad);
  std::printf("%-28s %s nnz %u max_seg %u: %s\n", name, f64 ? "f64" : "u64", A.nnz, L.max_seg,
              g_err == before ? "ok" : "FAILED");
}

int main() {
  std::vector<std::pair<const char*, HostCSR>> cases;
  {
    HostCSR c3;  // C3 shape at 2^18 rows (the stripe generator, 2^20 columns)
    const uint32_t n = 1u << 18, cols = 1u << 20, k = 32;
    c3.rows = n;
    c3.cols = cols;
    c3.nnz = n * k;
    c3.rowptr.resize(n + 1);
    c3.colind.resize(c3.nnz);
    std::vector<double> v(c3.nnz);
    genStripeCSR(0, n, cols, k, 1, 2, c3.rowptr.data(), c3.colind.data(), v.data());
    c3.vals.resize(c3.nnz);
    for (uint32_t i = 0; i < c3.nnz; ++i) c3.vals[i] = splitmix64_at(4, i);
    cases.emplace_back("stripe 2^18 x 2^20, 32/row", std::move(c3));
  }
  cases.emplace_back("random 20000 x 7937", random_csr(20000, 7937, 12, 1, 0));
  cases.emplace_back("random 16385 x 13001 dup", random_csr(16385, 13001, 16, 2, 1));
  cases.emplace_back("random 3000 x 20001", random_csr(3000, 20001, 40, 3, 0));
  cases.emplace_back("random 70001 x 8000", random_csr(70001, 8000, 6, 4, 1));
  for (auto& c : cases) {
    check_case<uint64_t>(c.first, c.second, false);
    check_case<double>(c.first, c.second, true);
  }
  std::printf("%s: %d violations\n", g_err ? "FAILED" : "ok", g_err);
  return g_err ? 1 : 0;
}
