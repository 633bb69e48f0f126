// vc_sim: CPU transliteration of k_vcache's addressing (csrc/vcache.hip) for
// checking the kernel's index math on the host.
//
// For one matrix it builds the product layout (csrc/plan.cpp build_vcache),
// then replays every work unit the way the kernel's two wave roles do --
// loader lanes' clamped x-pair loads and LDS stores (with the odd-cols patch),
// compute lanes' clamped quad loads, the DE-deep entry ring, the EPT register
// window and the overflow loop, the run continuation, the split combine -- with
// a bounds check on every global and LDS access and a check that no two lanes
// write the same LDS y row within one panel step (the kernel's no-race
// premise).  The result is compared bit-for-bit (ordered geometry) or within
// the FAST bound (split) with a sequential CSR reference.
//
// Test infrastructure (tests/test_vcache_sim.py); not part of the product.
//   g++ -O2 -std=c++17 -Icsrc -I../include tools/vc_sim.cpp csrc/plan.cpp host/Synthetic.cpp -o lib/vc_sim
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "../host/Synthetic.h"
#include "hipspmv_internal.h"
#include "vc_map.h"

#include <atomic>
#include <thread>

using namespace hipspmv;

static thread_local int g_errors = 0;  // per replay thread (main runs the cases in parallel)
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      if (g_errors++ < 20) {                               \
        std::fprintf(stderr, "VIOLATION %s:%d: ", __FILE__, __LINE__); \
        std::fprintf(stderr, __VA_ARGS__);                 \
        std::fprintf(stderr, "\n");                        \
      }                                                    \
    }                                                      \
  } while (0)

template <typename T>
struct Buf {  // bounds-checked global array
  const char* name;
  std::vector<T> v;
  Buf(const char* n, std::vector<T> src) : name(n), v(std::move(src)) {}
  template <class A>
  Buf(const char* n, const std::vector<T, A>& src) : name(n), v(src.begin(), src.end()) {}
  T get(size_t i) const {
    CHECK(i < v.size(), "%s[%zu] read, size %zu", name, i, v.size());
    return i < v.size() ? v[i] : T();
  }
  void put(size_t i, T x) {
    CHECK(i < v.size(), "%s[%zu] write, size %zu", name, i, v.size());
    if (i < v.size()) v[i] = x;
  }
};

// kernel configuration mirrored from vcache.hip VcCfg<SPLIT>
struct Cfg {
  int VR, VP, WL, DE, EPT, SPLIT;
  int LD = 0;  // 0: register-staged x loader, 1: LDS-DMA loader, 2: k_wgather (x gathered from global)
  int CB = 16; // column bits of the entry code
  int CX = 0;   // 1/2: cross-lane run continuation (needs every segment in the register window)
};

// sort_segments_by_line's specification: each segment's row runs stably
// sorted by the x line (column >> 4) of their first entry
static void ref_sort_by_line(VcacheLayout& L) {
  const uint32_t colmask = (1u << L.geom.colbits) - 1, units = L.nblocks * (uint32_t)L.geom.split;
  for (uint32_t u = 0; u < units; ++u)
    for (uint32_t i = 0; i < L.npad; ++i) {
      const uint32_t s0 = L.seg[(size_t)u * (L.npad + 1) + i], s1 = L.seg[(size_t)u * (L.npad + 1) + i + 1];
      std::vector<std::vector<std::pair<uint32_t, uint64_t>>> runs;
      std::vector<uint32_t> keys;
      for (uint32_t e = s0; e < s1; ++e) {
        if (e == s0 || !(L.code[e] & kVcCont)) {
          runs.emplace_back();
          keys.push_back((L.code[e] & colmask) >> 4);
        }
        runs.back().emplace_back(L.code[e], L.vals[e]);
      }
      std::vector<size_t> ord(runs.size());
      for (size_t k = 0; k < ord.size(); ++k) ord[k] = k;
      std::stable_sort(ord.begin(), ord.end(), [&](size_t p, size_t q) { return keys[p] < keys[q]; });
      uint32_t d = s0;
      for (size_t k : ord)
        for (auto& cv : runs[k]) {
          L.code[d] = cv.first;
          L.vals[d++] = cv.second;
        }
    }
}

static double madd(double acc, double a, double b) {
  volatile double p = a * b;  // rounded product, then the add (no contraction)
  return acc + p;
}

// Replays k_vcache for every unit; returns y.
// arrival_rev: the column parts of every block arrive in reverse unit order
// (the combine's result must not depend on the order)
static std::vector<double> simulate(const HostCSR& A, const VcacheLayout& L, const Cfg& c, const std::vector<double>& x,
                                    const std::vector<double>& yin, int beta, bool arrival_rev = false,
                                    const std::vector<uint64_t>* xmask = nullptr) {
  const bool gather = c.LD == 2;  // k_wgather: every wave computes, no loader role
  const int VT = 1024, NW = VT / 64, WC = gather ? NW : NW - c.WL, LT = c.WL * 64, CT = WC * 64;
  const uint32_t CMASK = (1u << c.CB) - 1, RMASK = (1u << (30 - c.CB)) - 1;
  const uint32_t PAIRS = c.VP / 2;
  const int NJ = LT ? (int)((PAIRS + LT - 1) / LT) : 0;
  const uint32_t rows = A.rows, cols = A.cols, nblocks = L.nblocks, npanels = L.npanels, part = L.part_panels,
                 npad = L.npad, rpb = L.rows_per_block, last = (uint32_t)L.code.size() - 1;
  Buf<uint32_t> seg{"seg", L.seg}, code{"ecode", L.code};
  Buf<double> vals{"evals", {}}, X{"x", x}, Yin{"y_in", yin}, Y{"y_out", std::vector<double>(rows, NAN)};
  vals.v.resize(L.vals.size());
  std::memcpy(vals.v.data(), L.vals.data(), 8 * L.vals.size());
  // k_vcache's partial layout: part q of block b at (q * nblocks + b) * VRP, VRP = VR rounded up to even
  const uint32_t VRP = (uint32_t)(c.VR + 1) & ~1u;
  Buf<double> partial{"partial", std::vector<double>((size_t)VRP * nblocks * c.SPLIT, NAN)};
  std::vector<uint32_t> tickets(nblocks, 0);
  const uint32_t units = nblocks * c.SPLIT;
  std::vector<std::vector<double>> ylds_of(units);
  std::vector<uint32_t> b_of(units), h_of(units);
  for (uint32_t bid = 0; bid < units; ++bid) {
    uint32_t b = bid, h = 0;
    if (c.SPLIT > 1) {
      const uint32_t g = bid / (8 * c.SPLIT), rem = bid % (8 * c.SPLIT);
      const uint32_t nbg = std::min(8u, nblocks - g * 8);
      h = rem / nbg;
      b = g * 8 + rem % nbg;
    }
    CHECK(b < nblocks && h < (uint32_t)c.SPLIT, "unit %u maps to (%u,%u)", bid, b, h);
    b_of[bid] = b;
    h_of[bid] = h;
    const uint32_t r0 = b * rpb;
    CHECK(r0 < rows, "unit %u r0 %u >= rows", bid, r0);
    const uint32_t nr = std::min(rpb, rows - r0);
    CHECK(nr <= (uint32_t)c.VR, "nr %u > VR", nr);
    const uint32_t p0 = vc_part_first(h, npanels, c.SPLIT);
    CHECK(p0 < npanels, "p0 %u >= npanels %u", p0, npanels);
    const uint32_t npu = vc_part_first(h + 1, npanels, c.SPLIT) - p0;
    CHECK(npu >= 1 && npu <= part && npad + 1 <= (uint32_t)L.geom.segmax, "npu %u part %u npad %u", npu, part, npad);
    std::vector<uint32_t> segl(L.geom.segmax, 0xDEADBEEF);
    for (uint32_t t = 0; t <= npad; ++t) segl[t] = seg.get(((size_t)b * c.SPLIT + h) * (npad + 1) + t);
    std::vector<double> ylds(c.VR, NAN);
    for (uint32_t i = 0; i < nr; ++i) ylds[i] = (beta && h == 0) ? Yin.get(r0 + i) : 0.0;
    const uint32_t cmax = (cols - 2) & ~1u;
    const double xlast = X.get(cols - 1);
    // loader: the LDS image of x panel s (load_x + store_x)
    auto panel = [&](uint32_t s) {
      std::vector<double> xb(gather ? 0 : c.VP, NAN);
      const uint32_t base = (p0 + std::min(s, npu - 1)) * c.VP;
      if (gather) return xb;  // x read from global at use (xat)
      if (c.LD == 1) {  // dma_x + patch_x: wave wl, instruction j, lane -> chunk (j*WL + wl)*64 + lane
        const int NDMA = (PAIRS + LT - 1) / LT;
        int patched = 0;
        for (int wl = 0; wl < c.WL; ++wl)
          for (int j = 0; j < NDMA; ++j)
            for (uint32_t lane = 0; lane < 64; ++lane) {
              const uint32_t c0 = (j * c.WL + wl) * 64, ch = c0 + lane;
              if (ch >= PAIRS) continue;
              const uint32_t a = std::min(base + 2 * ch, cmax);
              const uint32_t dst = 2 * c0 + 2 * lane;  // wave-uniform base + lane * 16 B
              CHECK(dst + 1 < (uint32_t)c.VP, "dma LDS dst %u", dst);
              xb[dst] = X.get(a);
              xb[dst + 1] = X.get(a + 1);
            }
        if ((cols & 1) && p0 + s == npanels - 1) {
          const uint32_t sl = cols - 1 - (p0 + s) * c.VP, ch = sl >> 1;
          for (int wl = 0; wl < c.WL; ++wl)
            for (uint32_t lane = 0; lane < 64; ++lane)
              if (ch < PAIRS && (ch / 64) % c.WL == (uint32_t)wl && (ch & 63) == lane) {
                CHECK(sl < (uint32_t)c.VP, "odd patch slot %u", sl);
                xb[sl] = xlast;
                ++patched;
              }
          CHECK(patched == 1, "odd patch applied %d times", patched);
        }
        return xb;
      }
      for (int t = 0; t < LT; ++t)
        for (int j = 0; j < NJ; ++j) {
          // the ordered loaders' x-line mask (build_xmask): a lane of an unused line loads nothing and
          // its LDS slot keeps what it held (NaN here: any read of it shows in y)
          if (xmask) {
            const uint64_t m = (*xmask)[((size_t)b * npanels + p0 + std::min(s, npu - 1)) * c.WL + t / 64];
            if (!((m >> (j * 8 + (t % 64) / 8)) & 1u)) continue;
          }
          const uint32_t a = std::min(base + 2 * (t + j * LT), cmax);
          const double v0 = X.get(a), v1 = X.get(a + 1);
          if ((j + 1) * LT <= (int)PAIRS || (uint32_t)(t + j * LT) < PAIRS) {
            const uint32_t slot = 2 * (t + j * LT);
            CHECK(slot + 1 < (uint32_t)c.VP, "x LDS slot %u", slot);
            xb[slot] = v0;
            xb[slot + 1] = v1;
          }
        }
      if ((cols & 1) && p0 + s == npanels - 1) {
        const uint32_t slot = cols - 1 - (p0 + s) * c.VP;
        CHECK(slot < (uint32_t)c.VP, "odd patch slot %u", slot);
        xb[slot] = xlast;
      }
      return xb;
    };
    for (uint32_t s = 0; s < npu; ++s) {
      const std::vector<double> xsv = panel(s);
      const uint64_t wbase = (uint64_t)(p0 + s) * c.VP;
      auto xs_at = [&](uint32_t col) {
        if (gather) {
          CHECK(wbase + col < cols, "gather x[%llu] beyond cols %u", (unsigned long long)(wbase + col), cols);
          return X.get(wbase + col);
        }
        CHECK(col < (uint32_t)c.VP, "x LDS col %u", col);
        return xsv[col];
      };
      const uint32_t beg = segl[s], end = segl[s + 1];
      CHECK(beg <= end, "segment %u [%u,%u)", s, beg, end);
      std::set<uint32_t> written;  // y rows written this step (race check)
      const uint32_t lbeg = segl[std::min(s, npad)];  // load_e(s), issued DE steps earlier
      if (c.CX) {  // apply_cx: products by every valid lane, continuations from lanes lw+k of the wave
        CHECK(end - beg <= (uint32_t)(c.EPT * CT), "segment %u of unit %u exceeds the register window", s, bid);
        std::vector<uint32_t> cc((size_t)CT * c.EPT);
        std::vector<double> pp((size_t)CT * c.EPT, 0.0);
        for (int ct = 0; ct < CT; ++ct)
          for (int j = 0; j < c.EPT; ++j) {
            const uint32_t i = std::min(lbeg + ct + j * CT, last);
            const uint32_t ei = beg + ct + j * CT;
            cc[(size_t)j * CT + ct] = code.get(i);
            if (ei < end) {
              CHECK(i == ei, "prefetched entry %u != used entry %u", i, ei);
              volatile double pr = vals.get(i) * xs_at(cc[(size_t)j * CT + ct] & CMASK);
              pp[(size_t)j * CT + ct] = pr;
            }
          }
        for (int j = 0; j < c.EPT; ++j)
          for (int ct = 0; ct < CT; ++ct) {
            const uint32_t ei = beg + ct + j * CT, cd0 = cc[(size_t)j * CT + ct];
            if (!(ei < end) || (cd0 & kVcCont)) continue;
            const uint32_t row = (cd0 >> c.CB) & RMASK;
            CHECK(row < nr, "row_local %u >= nr %u", row, nr);
            CHECK(!written.count(row), "race: row %u twice in step %u of unit %u", row, s, bid);
            written.insert(row);
            double acc = ylds[row] + pp[(size_t)j * CT + ct];
            bool more = (cd0 & kVcMore) != 0;
            for (uint32_t k = 1; more; ++k) {
              if ((uint32_t)(ct & 63) + k < 64) {
                const uint32_t nb = (uint32_t)ct + k, ni = beg + nb + j * CT, nc = cc[(size_t)j * CT + nb];
                CHECK(nb < (uint32_t)CT && ni == ei + k && ni < end && (nc & kVcCont),
                      "continuation lane %u: entry %u code %08x", nb, ni, nc);
                acc = acc + pp[(size_t)j * CT + nb];
                more = (nc & kVcMore) != 0;
              } else {  // scalar fallback from memory
                uint32_t i = ei + k, cd;
                do {
                  cd = code.get(i);
                  CHECK(i < end && (cd & kVcCont), "fallback entry %u", i);
                  volatile double pr = vals.get(i) * xs_at(cd & CMASK);
                  acc = acc + pr;
                  ++i;
                } while (cd & kVcMore);
                more = false;
              }
            }
            ylds[row] = acc;
          }
        continue;
      }
      for (int ct = 0; ct < CT; ++ct) {
        std::vector<uint32_t> cc(c.EPT);
        std::vector<double> vv(c.EPT);
        for (int j = 0; j < c.EPT; ++j) {  // branch-free clamped loads
          const uint32_t i = std::min(lbeg + ct + j * CT, last);
          cc[j] = code.get(i);
          vv[j] = vals.get(i);
        }
        for (int j = 0; j < c.EPT; ++j) {
          const uint32_t ei = beg + ct + j * CT;
          const bool act = ei < end && !(cc[j] & kVcCont);
          if (!act) continue;
          const uint32_t row = (cc[j] >> c.CB) & RMASK, col = cc[j] & CMASK;
          CHECK(row < nr, "row_local %u >= nr %u (unit %u step %u)", row, nr, bid, s);
          CHECK(col < (uint32_t)c.VP, "col_local %u", col);
          CHECK(!written.count(row), "race: row %u written twice in step %u of unit %u", row, s, bid);
          written.insert(row);
          double acc = madd(ylds[row], vv[j], xs_at(col));
          if (cc[j] & kVcMore) {
            uint32_t i = ei, cd = cc[j];
            do {
              ++i;
              cd = code.get(i);
              acc = madd(acc, vals.get(i), xs_at(cd & CMASK));
            } while (cd & kVcMore);
          }
          ylds[row] = acc;
        }
        for (uint32_t q = beg + c.EPT * CT + ct; q < end; q += CT) {  // overflow
          uint32_t cd = code.get(q);
          if (cd & kVcCont) continue;
          const uint32_t row = (cd >> c.CB) & RMASK;
          CHECK(row < nr && !written.count(row), "overflow row %u", row);
          written.insert(row);
          double acc = madd(ylds[row], vals.get(q), xs_at(cd & CMASK));
          uint32_t i = q;
          while (cd & kVcMore) {
            ++i;
            cd = code.get(i);
            acc = madd(acc, vals.get(i), xs_at(cd & CMASK));
          }
          ylds[row] = acc;
        }
      }
    }
    if (c.SPLIT == 1) {
      for (uint32_t i = 0; i < nr; ++i) Y.put(r0 + i, ylds[i]);
    } else {
      ylds_of[bid] = ylds;
    }
  }
  if (c.SPLIT > 1) {
    // ticket-first combine, arrivals in `order`: the first SPLIT-1 arrivals of a
    // block publish their partial; the last reads the others' (unwritten ones
    // are NaN and fail the comparison) and writes p0 + p1 (+ p2 + p3)
    std::vector<uint32_t> order(units), published(nblocks, 0);
    for (uint32_t i = 0; i < units; ++i) order[i] = arrival_rev ? units - 1 - i : i;
    for (uint32_t bid : order) {
      const uint32_t b = b_of[bid], h = h_of[bid];
      const uint32_t r0 = b * rpb, nr = std::min(rpb, rows - r0);
      if (tickets[b]++ != (uint32_t)c.SPLIT - 1) {
        for (uint32_t i = 0; i < nr; ++i) partial.put(((size_t)h * nblocks + b) * VRP + i, ylds_of[bid][i]);
        ++published[b];
        continue;
      }
      CHECK(published[b] == (uint32_t)c.SPLIT - 1, "block %u combined with %u partials published", b, published[b]);
      for (uint32_t i = 0; i < nr; ++i) {
        double acc = 0;
        for (int q = 0; q < c.SPLIT; ++q) {
          const double v = (uint32_t)q == h ? ylds_of[bid][i] : partial.get(((size_t)q * nblocks + b) * VRP + i);
          acc = q == 0 ? v : acc + v;
        }
        Y.put(r0 + i, acc);
      }
    }
    for (uint32_t b = 0; b < nblocks; ++b)
      CHECK(tickets[b] == (uint32_t)c.SPLIT, "block %u tickets %u", b, tickets[b]);
  }
  return Y.v;
}

static std::vector<double> reference(const HostCSR& A, const std::vector<double>& x, const std::vector<double>& yin,
                                     int beta) {
  std::vector<double> y(A.rows);
  for (uint32_t r = 0; r < A.rows; ++r) {
    double acc = beta ? yin[r] : 0.0;
    for (uint32_t e = A.rowptr[r]; e < A.rowptr[r + 1]; ++e) {
      double v;
      std::memcpy(&v, &A.vals[e], 8);
      acc = madd(acc, v, x[A.colind[e]]);
    }
    y[r] = acc;
  }
  return y;
}

static HostCSR random_csr(uint32_t rows, uint32_t cols, double density, uint64_t seed, bool long_row) {
  HostCSR A;
  A.rows = rows;
  A.cols = cols;
  A.rowptr.assign(rows + 1, 0);
  uint64_t k = 0;
  for (uint32_t r = 0; r < rows; ++r) {
    const bool empty = (splitmix64_at(seed, 1000000 + r) % 7) == 0;
    for (uint32_t c0 = 0; c0 < cols; ++c0) {
      const double u = (double)(splitmix64_at(seed, (uint64_t)r * cols + c0) >> 11) * 0x1.0p-53;
      if ((!empty && u < density) || (long_row && r == rows / 2)) {
        A.colind.push_back(c0);
        const double v = uniform11(splitmix64_at(seed + 1, k++));
        uint64_t bits;
        std::memcpy(&bits, &v, 8);
        A.vals.push_back(bits);
      }
    }
    A.rowptr[r + 1] = (uint32_t)A.colind.size();
  }
  A.nnz = (uint32_t)A.colind.size();
  return A;
}

// Slot -> unit mappings (csrc/vc_map.h): bijections onto the units, and
// MAP 1 keeps each column part on its own XCDs.
template <int SPLIT>
static int check_maps() {
  int bad = 0;
  for (uint32_t nb = 1; nb <= 300; ++nb) {
    for (int map = 0; map < 3; ++map) {
      if (map == 1 && !vc_map1_applies<SPLIT>(nb)) continue;
      std::vector<int> seen((size_t)nb * SPLIT, 0);
      for (uint32_t slot = 0; slot < nb * SPLIT; ++slot) {
        uint32_t b = 0, h = 0;
        if (map == 2)
          vc_unit_map2(slot, nb * SPLIT, nb, b, h);
        else if (map)
          vc_unit_map1<SPLIT>(slot, b, h);
        else
          vc_unit_map0<SPLIT>(slot, nb, b, h);
        if (b >= nb || h >= (uint32_t)SPLIT) {
          ++bad;
          continue;
        }
        seen[(size_t)b * SPLIT + h]++;
        if (map == 1 && h != (slot % 8) / (8 / SPLIT)) ++bad;  // part h on XCDs of group h
      }
      for (int c : seen) bad += c != 1;
    }
  }
  std::printf("unit mappings split=%d: %s\n", SPLIT, bad ? "FAIL" : "ok");
  return bad != 0;
}

int main(int argc, char** argv) {
  // cases: stripe C3-like (scaled), random ragged, odd cols, a long row
  struct Case {
    std::string name;
    HostCSR A;
  };
  std::vector<Case> cases;
  const int big = argc > 1 ? std::atoi(argv[1]) : 16;
  // "small": only the scaled stripe, R-MAT and random cases (sanitizer builds)
  const bool small = argc > 2 && std::string(argv[2]) == "small";
  {
    const uint32_t n = 1u << big, k = 32;
    HostCSR A;
    A.rows = A.cols = n;
    A.nnz = n * k;
    A.rowptr.resize(n + 1);
    A.colind.resize(A.nnz);
    std::vector<double> v(A.nnz);
    genStripeCSR(0, n, n, k, 1, 2, A.rowptr.data(), A.colind.data(), v.data());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"stripe 2^" + std::to_string(big), std::move(A)});
  }
  // row shards of the 2^20-column stripe matrix, as the row-partition and
  // golden-vector GPU tests create them (tests/test_golden_vectors.py)
  for (const uint32_t shard : {43691u, 65536u}) {
    if (small) break;
    const uint32_t n = shard, cols = 1u << 20, k = 32;
    HostCSR A;
    A.rows = n;
    A.cols = cols;
    A.nnz = n * k;
    A.rowptr.resize(n + 1);
    A.colind.resize(A.nnz);
    std::vector<double> v(A.nnz);
    genStripeCSR(43690, n, cols, k, 1, 2, A.rowptr.data(), A.colind.data(), v.data());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"stripe shard " + std::to_string(n) + "x2^20", std::move(A)});
  }
  {
    std::vector<uint32_t> rp, ci;
    std::vector<double> v;
    genRmatCSR(14, 16, 4, 0.57, 0.19, 0.19, rp, ci, v);
    HostCSR A;
    A.rows = A.cols = 1u << 14;
    A.nnz = (uint32_t)ci.size();
    A.rowptr.assign(rp.begin(), rp.end());
    A.colind.assign(ci.begin(), ci.end());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"rmat s14", std::move(A)});
  }
  // wide x (32 gather windows) and tall (more than 256 row blocks of 8192)
  for (const auto& shp : {std::array<uint32_t, 3>{20000, 1u << 22, 32}, std::array<uint32_t, 3>{2200001, 5003, 1}}) {
    if (small) break;
    const uint32_t n = shp[0], cols = shp[1], k = shp[2];
    HostCSR A;
    A.rows = n;
    A.cols = cols;
    A.nnz = n * k;
    A.rowptr.resize(n + 1);
    A.colind.resize(A.nnz);
    std::vector<double> v(A.nnz);
    genStripeCSR(7, n, cols, k, 1, 2, A.rowptr.data(), A.colind.data(), v.data());
    A.vals.resize(A.nnz);
    std::memcpy(A.vals.data(), v.data(), 8ull * A.nnz);
    cases.push_back({"stripe " + std::to_string(n) + "x" + std::to_string(cols), std::move(A)});
  }
  cases.push_back({"random 3000x20001", random_csr(3000, 20001, 0.002, 7, true)});
  // 4 panels of 4000 for the 3-part split: parts of 1, 1 and 2 panels (a ceil
  // cut used to leave the last part empty and the geometry ineligible)
  cases.push_back({"random 2000x14001", random_csr(2000, 14001, 0.003, 17, true)});
  cases.push_back({"random 5000x333", random_csr(5000, 333, 0.12, 9, false)});
  cases.push_back({"random 257x12161 dense rows", random_csr(257, 12161, 0.3, 11, true)});
  cases.push_back({"random 70000x13001", random_csr(70000, 13001, 0.0008, 13, false)});
  // must match VcCfg<1>/VcCfg<3> in csrc/vcache.hip (WL, DE, EPT); the split product: 3 LDS-DMA loaders,
  // cross-lane run continuation (CX 2 here models the kernel's xlane 3: same arithmetic, padded loops)
  const Cfg cfgs[] = {{kVcOrdered.rows, kVcOrdered.panel, 8, 4, 3, 1, 0},
                      {kVcSplit.rows, kVcSplit.panel, 3, 4, 2, 3, 1, 16, 2},
                      {kVcSplit4.rows, kVcSplit4.panel, 2, 4, 2, 4, 0},
                      {kVcOrdered.rows, kVcOrdered.panel, 8, 4, 3, 1, 1},
                      {kVcSplit.rows, kVcSplit.panel, 3, 4, 2, 3, 1},
                      {kVcSplit4.rows, kVcSplit4.panel, 2, 4, 2, 4, 1},
                      {kWgWindow.rows, kWgWindow.panel, 0, 4, 2, 1, 2, kWgWindow.colbits},
                      {kVcOrdered.rows, kVcOrdered.panel, 8, 4, 3, 1, 0, 16, 2},
                      {kVcSplit.rows, kVcSplit.panel, 6, 4, 3, 3, 0, 16, 2},
                      {kVcSplit.rows, kVcSplit.panel, 3, 4, 2, 3, 1, 16, 1},
                      {kVcSplit4.rows, kVcSplit4.panel, 2, 4, 2, 4, 0, 16, 2},
                      {kVcSplit4.rows, kVcSplit4.panel, 2, 4, 2, 4, 1, 16, 2},
                      {kWgWindow.rows, kWgWindow.panel, 0, 4, 4, 1, 2, kWgWindow.colbits, 2},
                      // k_wgather_split: the window layout in two column halves (kWgSplit)
                      {kWgSplit.rows, kWgSplit.panel, 0, 4, 3, 2, 2, kWgSplit.colbits}};
  int failures = check_maps<1>() + check_maps<2>() + check_maps<3>() + check_maps<4>();
  {  // the round-1 incident geometry: the ordered (split 1) kernel launched with the split layout's
     // 8192-row blocks -- 256 blocks over 2^20 rows, 128 of them past the last row -- is rejected,
     // as is any grid with a surplus block or a block taller than the kernel's LDS y block
    const uint32_t n = 1u << 20, np = (n + kVcOrdered.panel - 1) / kVcOrdered.panel;
    const bool incident = vcache_grid_ok(n, n, 8192, 256, np, np, np, kVcOrdered.panel, 1, kVcOrdered);
    const bool surplus = vcache_grid_ok(n, n, 4096, 257, np, np, np, kVcOrdered.panel, 1, kVcOrdered);
    const bool good = vcache_grid_ok(n, n, 4096, 256, np, np, np, kVcOrdered.panel, 1, kVcOrdered);
    const uint32_t nps = (n + kVcSplit.panel - 1) / kVcSplit.panel, part = (nps + 2) / 3;
    const uint32_t rs = (n + 84) / 85;  // the product split layout: 85 blocks x 3 parts
    const bool split_wrong_kernel = vcache_grid_ok(n, n, rs, 85, nps, part, part, kVcSplit.panel, 3, kVcOrdered);
    const bool split_good = vcache_grid_ok(n, n, rs, 85, nps, part, part, kVcSplit.panel, 3, kVcSplit);
    const bool ok = !incident && !surplus && good && !split_wrong_kernel && split_good;
    std::printf("grid guard (incident geometry rejected, product accepted): %s\n", ok ? "ok" : "FAIL");
    failures += !ok;
  }
  // the cases replay in parallel (a case's lines are printed together, in case order)
  std::vector<std::string> outs(cases.size());
  std::atomic<int> fails{failures};
  std::atomic<size_t> next{0};
  auto run_case = [&](Case& cs, std::string& text) {
    char* buf = nullptr;
    size_t len = 0;
    FILE* fo = open_memstream(&buf, &len);
    int nfail = 0;
    // host-side planning beside the replay: CSC -> CSR (csc_to_csr, the
    // hipspmv_create path) reproduces the case's CSR exactly, and the
    // csr_vector row groups tile the rows
    {
      const HostCSR& A = cs.A;
      std::vector<uint32_t> colptr(A.cols + 1, 0), rowind(A.nnz), cur;
      std::vector<uint64_t> cv(A.nnz);
      for (uint32_t e = 0; e < A.nnz; ++e) colptr[A.colind[e] + 1]++;
      for (uint32_t c = 0; c < A.cols; ++c) colptr[c + 1] += colptr[c];
      cur.assign(colptr.begin(), colptr.end() - 1);
      for (uint32_t r = 0; r < A.rows; ++r)
        for (uint32_t e = A.rowptr[r]; e < A.rowptr[r + 1]; ++e) {
          const uint32_t d = cur[A.colind[e]]++;
          rowind[d] = r | (e == A.rowptr[r] ? 1u << 31 : 0u);  // CMS marks are masked
          cv[d] = A.vals[e];
        }
      HostCSR B;
      std::string why;
      const int st = csc_to_csr(colptr.data(), rowind.data(), cv.data(), A.rows, A.cols, A.nnz, B, why);
      const bool same = st == 0 && B.rowptr == A.rowptr && B.colind == A.colind && B.vals == A.vals;
      std::vector<uint32_t> groups;
      build_row_groups(A, groups);
      bool tiles = groups.size() >= 2 && groups.front() == 0 && groups.back() == A.rows;
      for (size_t i = 1; i < groups.size(); ++i) {
        tiles = tiles && groups[i - 1] < groups[i];
        tiles = tiles && groups[i] - groups[i - 1] <= (uint32_t)kCvGroupRows;
        tiles = tiles && (groups[i - 1] / HIPSPMV_SHARD_ALIGN == (groups[i] - 1) / HIPSPMV_SHARD_ALIGN);
      }
      // a shard cut at multiples of HIPSPMV_SHARD_ALIGN has exactly the
      // unpartitioned matrix's groups over its rows (csr_vector bits do not
      // depend on the partition)
      bool shards = true;
      const uint32_t AL = HIPSPMV_SHARD_ALIGN;
      const uint32_t cuts[] = {0, A.rows / 3 / AL * AL, 2 * (A.rows / 3) / AL * AL, A.rows};
      for (int k = 0; k < 3; ++k) {
        const uint32_t s0 = cuts[k], s1 = cuts[k + 1];
        if (s1 <= s0) continue;
        HostCSR S;
        S.rows = s1 - s0;
        S.cols = A.cols;
        S.nnz = A.rowptr[s1] - A.rowptr[s0];
        S.rowptr.resize(S.rows + 1);
        for (uint32_t r = 0; r <= S.rows; ++r) S.rowptr[r] = A.rowptr[s0 + r] - A.rowptr[s0];
        std::vector<uint32_t> sg, want;
        build_row_groups(S, sg);
        for (uint32_t g : groups)
          if (g >= s0 && g <= s1) want.push_back(g - s0);
        shards = shards && sg == want;
      }
      // the wcsr segment matrix (build_windowed): each row's segments, read in
      // segidx order, are the row's entries in order; a segment lies in one
      // window; segments run window-major with rows ascending; groups tile it
      bool wins = true;
      // (and with a segment length cap: a row's pieces of one window are
      // consecutive, every piece but its last holds exactly cap entries)
      const std::pair<uint32_t, uint32_t> forms[] = {
          {8u, UINT32_MAX}, {12u, UINT32_MAX}, {kWcLog2Window, UINT32_MAX}, {8u, 3u}, {12u, 5u}};
      for (const bool by_line : {false, true})
      for (const auto& [lw, cap] : forms) {
        WinLayout W;
        build_windowed(A, lw, W, cap, by_line);
        const HostCSR& G = W.seg;
        wins = wins && G.rows == W.nseg && G.nnz == A.nnz && G.rowptr.size() == (size_t)W.nseg + 1 &&
               G.rowptr[0] == 0 && G.rowptr[W.nseg] == A.nnz && W.rowseg.size() == (size_t)A.rows + 1 &&
               W.rowseg[A.rows] == W.nseg && W.segidx.size() == W.nseg;
        if (!wins) break;
        std::vector<uint32_t> owner(W.nseg, UINT32_MAX);
        for (uint32_t r = 0; r < A.rows && wins; ++r) {
          uint32_t e = A.rowptr[r], prevw = 0;
          for (uint32_t k = W.rowseg[r]; k < W.rowseg[r + 1] && wins; ++k) {
            const uint32_t sg = W.segidx[k];
            wins = sg < W.nseg && owner[sg] == UINT32_MAX && G.rowptr[sg] < G.rowptr[sg + 1];
            if (!wins) break;
            owner[sg] = r;
            const uint32_t w = G.colind[G.rowptr[sg]] >> lw;
            const uint32_t prevlen = k == W.rowseg[r] ? 0 : G.rowptr[W.segidx[k - 1] + 1] - G.rowptr[W.segidx[k - 1]];
            // a row's segments in ascending windows (a full piece may continue in its window)
            wins = (k == W.rowseg[r] || w > prevw || (w == prevw && prevlen == cap)) &&
                   G.rowptr[sg + 1] - G.rowptr[sg] <= cap;
            prevw = w;
            for (uint32_t d = G.rowptr[sg]; d < G.rowptr[sg + 1] && wins; ++d, ++e)
              wins = e < A.rowptr[r + 1] && G.colind[d] == A.colind[e] && G.vals[d] == A.vals[e] &&
                     (G.colind[d] >> lw) == w;
          }
          wins = wins && e == A.rowptr[r + 1];
        }
        // window-major; in a window rows ascending, or (by_line) first-column
        // lines ascending and rows ascending within a line
        const uint32_t ksh = by_line && lw >= 4 ? 4 : lw;
        for (uint32_t sg = 1; sg < W.nseg && wins; ++sg) {
          const uint32_t k0 = G.colind[G.rowptr[sg - 1]] >> ksh, k1 = G.colind[G.rowptr[sg]] >> ksh;
          wins = k0 < k1 || (k0 == k1 && (owner[sg - 1] < owner[sg] ||
                                           (cap != UINT32_MAX && owner[sg - 1] == owner[sg])));
        }
        for (uint32_t w = 0; w + 1 < W.winseg.size() && wins; ++w)  // window w's segments, [winseg[w], winseg[w+1])
          for (uint32_t sg = W.winseg[w]; sg < W.winseg[w + 1] && wins; ++sg)
            wins = (G.colind[G.rowptr[sg]] >> lw) == w;
        std::vector<uint32_t> gg;
        build_row_groups(G, gg);
        wins = wins && gg.front() == 0 && gg.back() == G.rows;
        // the hot-column form (mark_hot_columns): every entry decodes to its column, slots < K, each
        // window's hot columns ascending, distinct and inside the window, and a hot column's count is
        // at least every cold column's of the window
        for (const uint32_t K : {1u, 16u}) {
          if (!wins) break;
          WinLayout H = W;
          std::vector<uint32_t> hot;
          wins = mark_hot_columns(H, K, hot) && hot.size() == (size_t)(W.winseg.size() - 1) * K;
          for (uint32_t w = 0; w + 1 < W.winseg.size() && wins; ++w) {
            const uint32_t e0 = G.rowptr[W.winseg[w]], e1 = G.rowptr[W.winseg[w + 1]];
            std::vector<uint32_t> cnt(1u << lw, 0);
            std::vector<char> is_hot(1u << lw, 0);
            uint32_t nh = 0;
            for (uint32_t e = e0; e < e1 && wins; ++e) {
              const uint32_t c = H.seg.colind[e];
              const uint32_t col = (c & kWcHotFlag) ? hot[(size_t)w * K + (c & ~kWcHotFlag)] : c;
              wins = col == G.colind[e] && ((c & kWcHotFlag) == 0 || (c & ~kWcHotFlag) < K);
              cnt[col & ((1u << lw) - 1)]++;
              if (c & kWcHotFlag) is_hot[col & ((1u << lw) - 1)] = 1;
            }
            uint32_t minhot = UINT32_MAX, maxcold = 0;
            for (uint32_t c = 0; c < (1u << lw); ++c) {
              if (is_hot[c]) minhot = std::min(minhot, cnt[c]), ++nh;
              else maxcold = std::max(maxcold, cnt[c]);
            }
            wins = wins && (nh == 0 || minhot >= maxcold) && nh <= K;
            for (uint32_t i = 1; i < nh && wins; ++i)
              wins = hot[(size_t)w * K + i - 1] < hot[(size_t)w * K + i] && (hot[(size_t)w * K + i] >> lw) == w;
          }
        }
      }
      nfail += !(same && tiles && shards && wins);
      std::fprintf(fo, "%-28s csc_to_csr %s, row groups %s, shard groups %s, windowed segments %s\n", cs.name.c_str(),
                  same ? "ok" : "FAIL", tiles ? "ok" : "FAIL", shards ? "ok" : "FAIL", wins ? "ok" : "FAIL");
    }
    std::vector<double> x(cs.A.cols), yin(cs.A.rows);
    for (uint32_t i = 0; i < cs.A.cols; ++i) x[i] = uniform11(splitmix64_at(3, i));
    for (uint32_t i = 0; i < cs.A.rows; ++i) yin[i] = uniform11(splitmix64_at(5, i));
    for (const Cfg& c : cfgs) {
      VcGeom g{c.VR, c.VP, c.SPLIT, c.CB};
      if (c.LD == 2) g.segmax = kWgWindow.segmax;  // k_wgather's segment table
      if (!vcache_eligible(cs.A, g)) {
        std::fprintf(fo, "%-28s split=%d ld=%d: not eligible\n", cs.name.c_str(), c.SPLIT, c.LD);
        continue;
      }
      VcacheLayout L;
      build_vcache(cs.A, g, L);
      if (c.LD == 2) {  // the wgather layout as hipspmv_create builds it; against a plain stable sort
        VcacheLayout R = L, D;
        ref_sort_by_line(R);
        sort_segments_by_line(L);
        build_vcache(cs.A, g, D, true);
        if (!(R.code == L.code && R.vals == L.vals && R.seg == L.seg && D.code == L.code && D.vals == L.vals &&
              D.seg == L.seg)) {
          std::fprintf(fo, "%-28s sort_segments_by_line differs from the stable-sort reference\n", cs.name.c_str());
          ++nfail;
        }
      }
      // the launcher's guard (vcache_grid_ok) accepts every product layout
      if (!vcache_grid_ok(cs.A.rows, cs.A.cols, L.rows_per_block, L.nblocks, L.npanels, L.part_panels, L.npad,
                          L.geom.panel, c.SPLIT, g)) {
        std::fprintf(fo, "%-28s split=%d: product layout REJECTED by vcache_grid_ok\n", cs.name.c_str(), c.SPLIT);
        ++nfail;
        continue;
      }
      if (c.CX && L.max_seg > (uint32_t)((16 - c.WL) * 64 * c.EPT)) {  // launch_vcache falls back to CX 0
        std::fprintf(fo, "%-28s split=%d cx=%d: segments exceed the window, CX 0 runs\n", cs.name.c_str(), c.SPLIT, c.CX);
        continue;
      }
      // the product's bank-aware placement (plan.cpp place_segments_banked):
      // a permutation inside every segment, runs consecutive inside one wave,
      // and the same result bits as the (row, column) layout
      VcacheLayout B;
      // the product layouts: split (xlane 3, modelled as CX 2) and the ordered geometry
      const bool banked = (c.SPLIT >= 3 && c.LD == 1 && c.CX >= 2) || (c.SPLIT == 1 && c.LD != 2);
      if (banked) {
        B = L;
        const uint32_t CT = (uint32_t)(16 - c.WL) * 64;
        place_segments_banked(B, CT);
        bool perm = B.seg == L.seg;
        const uint32_t units = L.nblocks * (uint32_t)c.SPLIT;
        for (uint32_t u = 0; u < units && perm; ++u)
          for (uint32_t i = 0; i < L.npad && perm; ++i) {
            const uint32_t s0 = L.seg[(size_t)u * (L.npad + 1) + i], s1 = L.seg[(size_t)u * (L.npad + 1) + i + 1];
            std::vector<std::pair<uint32_t, uint64_t>> a0, a1;
            for (uint32_t e = s0; e < s1; ++e) {
              a0.emplace_back(L.code[e], L.vals[e]);
              a1.emplace_back(B.code[e], B.vals[e]);
              if ((B.code[e] & kVcCont) && (e == s0 || !(B.code[e - 1] & kVcMore) ||
                                             (B.row_runs && (e - s0) % 16 == 0)))
                perm = false;  // a continuation right after its run's previous entry (row_runs: same DPP row)
            }
            std::sort(a0.begin(), a0.end());
            std::sort(a1.begin(), a1.end());
            perm = perm && a0 == a1;
          }
        if (!perm) {
          std::fprintf(fo, "%-28s place_segments_banked: not a run-preserving permutation\n", cs.name.c_str());
          ++nfail;
        }
      }
      for (int beta = 0; beta < 2; ++beta) {
        g_errors = 0;
        const auto y = simulate(cs.A, L, c, x, yin, beta);
        if (banked) {
          const auto yb = simulate(cs.A, B, c, x, yin, beta);
          if (std::memcmp(y.data(), yb.data(), 8ull * cs.A.rows) != 0) {
            std::fprintf(fo, "%-28s banked placement changes result bits\n", cs.name.c_str());
            ++nfail;
          }
          if (c.SPLIT == 1 && c.LD == 0 && c.WL == (int)kVcOrderedLoaders) {
            // the ordered loaders skipping the x lines no entry of a panel uses: the same bits
            std::vector<uint64_t> xm;
            build_xmask(B, kVcOrderedLoaders, xm);
            const auto ym = simulate(cs.A, B, c, x, yin, beta, false, &xm);
            size_t skipped = 0, total = 0;
            for (uint64_t w : xm) skipped += 64 - __builtin_popcountll(w), total += 64;
            if (std::memcmp(y.data(), ym.data(), 8ull * cs.A.rows) != 0) {
              std::fprintf(fo, "%-28s x-line mask changes result bits\n", cs.name.c_str());
              ++nfail;
            } else if (beta == 0) {
              std::fprintf(fo, "%-28s x-line mask: same bits, %.1f %% of line slots skipped\n", cs.name.c_str(),
                          100.0 * skipped / std::max<size_t>(total, 1));
            }
          }
        }
        const auto r = reference(cs.A, x, yin, beta);
        size_t bad = 0;
        if (c.SPLIT > 1) {  // deterministic: the other arrival order gives the same bits
          const auto y2 = simulate(cs.A, L, c, x, yin, beta, true);
          bad += std::memcmp(y.data(), y2.data(), 8ull * cs.A.rows) != 0;
        }
        for (uint32_t i = 0; i < cs.A.rows; ++i) {
          if (c.SPLIT == 1) {
            bad += std::memcmp(&y[i], &r[i], 8) != 0;
          } else {
            double absp = std::fabs(beta ? yin[i] : 0.0);
            uint32_t len = cs.A.rowptr[i + 1] - cs.A.rowptr[i];
            for (uint32_t e = cs.A.rowptr[i]; e < cs.A.rowptr[i + 1]; ++e) {
              double v;
              std::memcpy(&v, &cs.A.vals[e], 8);
              absp += std::fabs(v * x[cs.A.colind[e]]);
            }
            bad += !(std::fabs(y[i] - r[i]) <= 2.0 * (len + 1) * 0x1.0p-53 * absp + 1e-300);
          }
        }
        const bool ok = bad == 0 && g_errors == 0;
        nfail += !ok;
        std::fprintf(fo, "%-28s split=%d ld=%d cx=%d beta=%d units=%u panels=%u: %s (%zu rows off, %d violations)\n",
                    cs.name.c_str(), c.SPLIT, c.LD, c.CX, beta, L.nblocks * c.SPLIT, L.npanels, ok ? "ok" : "FAIL",
                    bad, g_errors);
      }
    }
      std::fclose(fo);
    text.assign(buf, len);
    std::free(buf);
    fails += nfail;
  };
  std::vector<std::thread> pool;
  const unsigned nt = std::max(1u, std::min<unsigned>(8, std::thread::hardware_concurrency()));
  for (unsigned t = 0; t < nt; ++t)
    pool.emplace_back([&] {
      for (size_t i; (i = next++) < cases.size();) run_case(cases[i], outs[i]);
    });
  for (auto& th : pool) th.join();
  for (const auto& o : outs) std::fputs(o.c_str(), stdout);
  failures = fails;
  return failures ? 1 : 0;
}
