// Host-side planning for libhipspmv: CSC -> CSR transpose, validation, and the
// device layouts each kernel reads.
#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "hipspmv.h"
#include "hipspmv_internal.h"

namespace hipspmv {

namespace {
constexpr uint32_t kRowMask = 0x3FFFFFFFu;  // SparseMatrix.cpp:64,77 cold-miss-skip bits

// fn(t, lo, hi) over nt contiguous chunks of [0, n), chunk 0 on the calling
// thread.  The builders allocate before they fork: a worker never throws.
template <class F>
void par_chunks(uint64_t n, unsigned nt, F&& fn) {
  nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, n));
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; ++t) ts.emplace_back([&fn, t, n, nt] { fn(t, n * t / nt, n * (t + 1) / nt); });
  fn(0u, (uint64_t)0, n / nt);
  for (auto& th : ts) th.join();
}

// row ranges of about nnz / nt entries each: rows [b[t], b[t+1])
std::vector<uint32_t> row_chunks(const uint32_t* rowptr, uint32_t rows, unsigned nt) {
  std::vector<uint32_t> b(nt + 1, rows);
  b[0] = 0;
  const uint64_t nnz = rowptr[rows];
  for (unsigned t = 1; t < nt; ++t) {
    const uint32_t target = (uint32_t)(nnz * t / nt);
    b[t] = (uint32_t)(std::lower_bound(rowptr, rowptr + rows + 1, target) - rowptr);
    b[t] = std::max(std::min(b[t], rows), b[t - 1]);
  }
  return b;
}

// fn(t, r0, r1) over entry-balanced row ranges, in parallel
template <class F>
void par_rows(const uint32_t* rowptr, uint32_t rows, F&& fn) {
  const unsigned nt = std::max(1u, std::min(plan_threads(), std::max(1u, rows / 64)));
  const std::vector<uint32_t> b = row_chunks(rowptr, rows, nt);
  par_chunks(nt, nt, [&](unsigned, uint64_t lo, uint64_t hi) {
    for (uint64_t t = lo; t < hi; ++t) fn((unsigned)t, b[t], b[t + 1]);
  });
}
}  // namespace

unsigned plan_threads() {
  for (const char* k : {"HIPSPMV_THREADS", "OMP_NUM_THREADS"})
    if (const char* e = std::getenv(k)) {
      const int v = std::atoi(e);
      if (v > 0) return (unsigned)std::min(v, 256);
    }
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Stable counting-sort transpose, the algorithm of software/csr2csc.c:11-39
// applied to the CSC arrays (so it yields CSR with column ids ascending within
// each row, and duplicate entries in their CSC order -- exactly the order in
// which SoftwareSpMV::exec (SoftwareSpMV.cpp:59-64) adds them into y[row]).
// In parallel: thread t owns a range of rows, counts and places only their
// entries while walking every column in order -- the same bytes as a serial
// transpose.
int csc_to_csr(const uint32_t* colptr, const uint32_t* rowind, const void* vals, uint32_t rows, uint32_t cols,
               uint32_t nnz, HostCSR& out, std::string& why) {
  if (colptr[0] != 0 || colptr[cols] != nnz) {
    why = "colptr[0] must be 0 and colptr[cols] must equal nnz";
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  for (uint32_t c = 0; c < cols; ++c)
    if (colptr[c + 1] < colptr[c]) {
      why = "colptr not monotone at column " + std::to_string(c);
      return HIPSPMV_ERR_INVALID_MATRIX;
    }
  const unsigned nt = std::max(1u, std::min(plan_threads(), std::max(1u, rows / 1024)));
  {  // the first out-of-range row id
    std::vector<uint64_t> bad(nt, UINT64_MAX);
    par_chunks(nnz, nt, [&](unsigned t, uint64_t lo, uint64_t hi) {
      for (uint64_t e = lo; e < hi; ++e)
        if ((rowind[e] & kRowMask) >= rows) {
          bad[t] = e;
          return;
        }
    });
    const uint64_t e = *std::min_element(bad.begin(), bad.end());
    if (e != UINT64_MAX) {
      why = "row id " + std::to_string(rowind[e] & kRowMask) + " out of range at element " + std::to_string(e);
      return HIPSPMV_ERR_INVALID_MATRIX;
    }
  }
  out.rows = rows;
  out.cols = cols;
  out.nnz = nnz;
  out.rowptr.resize((size_t)rows + 1);
  out.colind.resize(nnz);
  out.vals.resize(nnz);
  const uint64_t* v = static_cast<const uint64_t*>(vals);
  auto rlo = [&](uint64_t t) { return (uint32_t)((uint64_t)rows * t / nt); };
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {  // counts of the thread's rows
    for (uint64_t t = t0; t < t1; ++t) {
      const uint32_t r0 = rlo(t), span = rlo(t + 1) - r0;
      for (uint32_t r = r0; r < r0 + span; ++r) out.rowptr[r + 1] = 0;
      for (uint32_t e = 0; e < nnz; ++e) {
        const uint32_t r = (rowind[e] & kRowMask) - r0;
        if (r < span) out.rowptr[r0 + r + 1]++;
      }
    }
  });
  out.rowptr[0] = 0;
  for (uint32_t r = 0; r < rows; ++r) out.rowptr[r + 1] += out.rowptr[r];
  hvec<uint32_t> cursor(out.rowptr.begin(), out.rowptr.end() - 1);
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    for (uint64_t t = t0; t < t1; ++t) {
      const uint32_t r0 = rlo(t), span = rlo(t + 1) - r0;
      for (uint32_t c = 0; c < cols; ++c)
        for (uint32_t e = colptr[c]; e < colptr[c + 1]; ++e) {
          const uint32_t r = (rowind[e] & kRowMask) - r0;
          if (r < span) {
            const uint32_t d = cursor[r0 + r]++;
            out.colind[d] = c;
            out.vals[d] = v[e];
          }
        }
    }
  });
  return HIPSPMV_OK;
}

int copy_csr(const uint32_t* rowptr, const uint32_t* colind, const void* vals, uint32_t rows, uint32_t cols,
             uint32_t nnz, HostCSR& out, std::string& why) {
  if (rowptr[0] != 0 || rowptr[rows] != nnz) {
    why = "rowptr[0] must be 0 and rowptr[rows] must equal nnz";
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  for (uint32_t r = 0; r < rows; ++r)
    if (rowptr[r + 1] < rowptr[r]) {
      why = "rowptr not monotone at row " + std::to_string(r);
      return HIPSPMV_ERR_INVALID_MATRIX;
    }
  out.rows = rows;
  out.cols = cols;
  out.nnz = nnz;
  // the caller's arrays, read in place for the duration of the create call
  out.rowptr.borrow(rowptr, (size_t)rows + 1);
  out.colind.borrow(colind, nnz);
  out.vals.borrow(static_cast<const uint64_t*>(vals), nnz);
  // check the column ids
  const unsigned nt = plan_threads();
  std::vector<uint64_t> bad(nt, UINT64_MAX);
  par_chunks(nnz, nt, [&](unsigned t, uint64_t lo, uint64_t hi) {
    for (uint64_t e = lo; e < hi; ++e)
      if (colind[e] >= cols) {
        bad[t] = e;
        return;
      }
  });
  const uint64_t e = *std::min_element(bad.begin(), bad.end());
  if (e != UINT64_MAX) {
    why = "column id " + std::to_string(colind[e]) + " out of range at element " + std::to_string(e);
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
  return HIPSPMV_OK;
}

static uint32_t vcache_rows_per_block(uint32_t rows, const VcGeom& g) {
  // About one work unit per CU (256 CUs on MI355X), never more rows than the
  // LDS y budget; at least 64 rows so tiny matrices use few units.
  const uint32_t units = 256 / (uint32_t)g.split;  // blocks that fill the chip once
  uint32_t r = (uint32_t)(((uint64_t)rows + units - 1) / units);
  r = std::max<uint32_t>(r, 64);
  return std::min<uint32_t>(r, (uint32_t)g.rows);
}

void vcache_geometry(uint32_t rows, uint32_t cols, const VcGeom& g, VcacheLayout& out) {
  const uint32_t P = (uint32_t)g.panel, S = (uint32_t)g.split;
  out.geom = g;
  out.rows_per_block = vcache_rows_per_block(rows, g);
  out.nblocks = (rows + out.rows_per_block - 1) / out.rows_per_block;
  out.npanels = (cols + P - 1) / P;
  out.part_panels = (out.npanels + S - 1) / S;  // the largest part (vc_part_first cuts)
  out.npad = out.part_panels;                   // the kernel clamps prefetches past its last panel
}

bool vcache_eligible(const HostCSR& a, const VcGeom& g) {
  if (a.cols < 2 || a.rows == 0 || a.nnz == 0) return false;
  // the entry code must hold col_local and row_local
  if ((uint64_t)g.panel > (1ull << g.colbits) || (uint64_t)g.rows > (1ull << (30 - g.colbits))) return false;
  const uint32_t np = (a.cols + g.panel - 1) / g.panel;
  if (np < (uint32_t)g.split) return false;  // every column part owns >= 1 panel (vc_part_first)
  const uint32_t part = (np + g.split - 1) / g.split;
  const uint32_t npad = part;  // the kernel clamps prefetches past its last panel
  if (npad + 1 > (uint32_t)g.segmax) return false;
  // panel order must equal each row's summation order: columns non-decreasing
  std::atomic<bool> sorted{true};
  par_rows(a.rowptr.data(), a.rows, [&](unsigned, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1 && sorted.load(std::memory_order_relaxed); ++r)
      for (uint32_t e = a.rowptr[r] + 1; e < a.rowptr[r + 1]; ++e)
        if (a.colind[e] < a.colind[e - 1]) {
          sorted = false;
          return;
        }
  });
  return sorted;
}

// Longest run of one row inside one panel of `panel` columns (columns sorted
// within each row, as vcache_eligible requires): the kernels walk a run
// sequentially in one lane, so AUTO keeps matrices with long runs (R-MAT hub
// rows) off the vcache-family kernels.
uint32_t vcache_max_run(const HostCSR& a, uint32_t panel) {
  std::vector<uint32_t> best(plan_threads() + 1, 0);
  par_rows(a.rowptr.data(), a.rows, [&](unsigned t, uint32_t r0, uint32_t r1) {
    uint32_t b = 0;
    for (uint32_t r = r0; r < r1; ++r) {
      uint32_t run = 0, prev = UINT32_MAX;
      for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e) {
        const uint32_t p = a.colind[e] / panel;
        run = p == prev ? run + 1 : 1;
        prev = p;
        b = std::max(b, run);
      }
    }
    best[t] = b;
  });
  return *std::max_element(best.begin(), best.end());
}

// Row-run sort by x line (k_wgather's segment order, sort_segments_by_line)
namespace {
struct LineSort {
  uint32_t colmask, lo_bits, nlo, nhi;
  std::vector<uint32_t> key, start, len, o1, o2, clo, chi, code;
  std::vector<uint64_t> vals;
  explicit LineSort(uint32_t colbits) : colmask((1u << colbits) - 1) {
    const uint32_t kb = colbits > 4 ? colbits - 4 : 1;
    lo_bits = (kb + 1) / 2;
    nlo = 1u << lo_bits;
    nhi = 1u << (kb - lo_bits);
    clo.resize(nlo + 1);
    chi.resize(nhi + 1);
  }
  void operator()(uint32_t* C, uint64_t* V, uint32_t s0, uint32_t s1) {
    if (s1 - s0 < 2) return;
    key.clear();
    start.clear();
    len.clear();
    for (uint32_t e = s0; e < s1;) {
      uint32_t f = e + 1;
      while (f < s1 && (C[f] & kVcCont)) ++f;
      key.push_back((C[e] & colmask) >> 4);
      start.push_back(e - s0);
      len.push_back(f - e);
      e = f;
    }
    const uint32_t m = (uint32_t)key.size();
    o1.resize(m);
    o2.resize(m);
    std::fill(clo.begin(), clo.end(), 0u);  // pass 1: low bits (stable)
    for (uint32_t k = 0; k < m; ++k) clo[(key[k] & (nlo - 1)) + 1]++;
    for (uint32_t b = 0; b < nlo; ++b) clo[b + 1] += clo[b];
    for (uint32_t k = 0; k < m; ++k) o1[clo[key[k] & (nlo - 1)]++] = k;
    std::fill(chi.begin(), chi.end(), 0u);  // pass 2: high bits (stable)
    for (uint32_t k = 0; k < m; ++k) chi[(key[k] >> lo_bits) + 1]++;
    for (uint32_t b = 0; b < nhi; ++b) chi[b + 1] += chi[b];
    for (uint32_t k = 0; k < m; ++k) {
      const uint32_t r = o1[k];
      o2[chi[key[r] >> lo_bits]++] = r;
    }
    code.assign(C + s0, C + s1);
    vals.assign(V + s0, V + s1);
    uint32_t d = s0;
    for (uint32_t k = 0; k < m; ++k) {
      const uint32_t r = o2[k];
      for (uint32_t q = 0; q < len[r]; ++q, ++d) {
        C[d] = code[start[r] + q];
        V[d] = vals[start[r] + q];
      }
    }
  }
};
}  // namespace

// Entries of row block b that fall into column panel p form segment (b, p),
// ordered by (row, column); each row's entries keep their CSR order, so a
// thread that walks a row run in a segment, and the panels in ascending
// order, adds the row's products in ascending column order.  A work unit
// (b, h) covers panels [vc_part_first(h), vc_part_first(h+1)); its seg row
// lists npad+1 offsets (empty segments past its last panel).
void build_vcache(const HostCSR& a, const VcGeom& g, VcacheLayout& out, bool by_line) {
  const uint32_t P = (uint32_t)g.panel, S = (uint32_t)g.split;
  vcache_geometry(a.rows, a.cols, g, out);
  const uint32_t R = out.rows_per_block, nb = out.nblocks, np = out.npanels, npad = out.npad;
  out.seg.assign((size_t)nb * S * (npad + 1), 0);
  out.code.resize(a.nnz);
  out.vals.resize(a.nnz);
  // row blocks are independent (block b's entries start at rowptr[b R]):
  // contiguous block ranges per thread, entry-balanced
  const unsigned nt = std::max(1u, std::min(plan_threads(), nb));
  std::vector<uint32_t> bb(nt + 1, nb);
  bb[0] = 0;
  for (unsigned t = 1; t < nt; ++t) {
    const uint32_t target = (uint32_t)((uint64_t)a.nnz * t / nt);
    uint32_t b = (uint32_t)(std::lower_bound(a.rowptr.begin(), a.rowptr.end(), target) - a.rowptr.begin()) / R;
    bb[t] = std::max(std::min(b, nb), bb[t - 1]);
  }
  std::vector<uint32_t> tmax(nt, 0);
  std::vector<uint64_t> tcont(nt, 0);
  std::vector<std::vector<uint32_t>> tcnt(nt, std::vector<uint32_t>(np + 1)), tcur(nt, std::vector<uint32_t>(np));
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    LineSort sort((uint32_t)g.colbits);
    for (uint64_t t = t0; t < t1; ++t) {
      std::vector<uint32_t>& cnt = tcnt[t];
      std::vector<uint32_t>& cur = tcur[t];
      for (uint32_t b = bb[t]; b < bb[t + 1]; ++b) {
        const uint32_t r0 = b * R, r1 = std::min(a.rows, r0 + R), base = a.rowptr[r0];
        std::fill(cnt.begin(), cnt.end(), 0);
        for (uint32_t e = a.rowptr[r0]; e < a.rowptr[r1]; ++e) cnt[a.colind[e] / P + 1]++;
        for (uint32_t p = 0; p < np; ++p) {
          tmax[t] = std::max(tmax[t], cnt[p + 1]);
          cnt[p + 1] += cnt[p];
        }
        for (uint32_t h = 0; h < S; ++h) {
          uint32_t* seg = &out.seg[((size_t)b * S + h) * (npad + 1)];
          const uint32_t pfirst = vc_part_first(h, np, S), plast = vc_part_first(h + 1, np, S);
          for (uint32_t i = 0; i <= npad; ++i) seg[i] = base + cnt[std::min(pfirst + i, plast)];
        }
        std::copy(cnt.begin(), cnt.end() - 1, cur.begin());
        for (uint32_t r = r0; r < r1; ++r) {
          uint32_t prev_d = UINT32_MAX, prev_p = UINT32_MAX;
          for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e) {
            const uint32_t c = a.colind[e], p = c / P;
            const uint32_t d = base + cur[p]++;
            uint32_t code = (c - p * P) | ((r - r0) << g.colbits);
            if (p == prev_p && d == prev_d + 1) {  // same row, same segment, adjacent: extend the run
              code |= kVcCont;
              ++tcont[t];
              out.code[prev_d] |= kVcMore;
            }
            out.code[d] = code;
            out.vals[d] = a.vals[e];
            prev_d = d;
            prev_p = p;
          }
        }
        if (by_line)  // the block's segments while they are still in cache (sort_segments_by_line)
          for (uint32_t p = 0; p < np; ++p) sort(out.code.data(), out.vals.data(), base + cnt[p], base + cnt[p + 1]);
      }
    }
  });
  out.max_seg = *std::max_element(tmax.begin(), tmax.end());
  out.n_cont = 0;
  for (uint64_t c : tcont) out.n_cont += c;
  out.max_run = vcache_max_run(a, P);
}

// k_wgather's order inside each segment: row runs (a run is one row's entries
// in this window, consecutive, in column order) stably sorted by the 128-byte
// x line of their first column, so lanes of a wave that gather from one line
// sit next to each other and the gather instruction merges them into one L2
// request.  Rows stay one run per segment and keep their column order inside
// it: ORDERED sums are unchanged.  Per segment an LSD radix sort of the runs
// (two passes of half the line bits), buffers reused across segments.
void sort_segments_by_line(VcacheLayout& L) {
  const uint32_t units = L.nblocks * (uint32_t)L.geom.split, npad = L.npad;
  const unsigned nt = std::max(1u, std::min(plan_threads(), units));
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    LineSort sort((uint32_t)L.geom.colbits);
    for (uint64_t t = t0; t < t1; ++t)
      for (uint32_t u = (uint32_t)t; u < units; u += nt) {
        const uint32_t* sg = &L.seg[(size_t)u * (npad + 1)];
        for (uint32_t i = 0; i < npad; ++i) sort(L.code.data(), L.vals.data(), sg[i], sg[i + 1]);
      }
  });
}

// LDS-bank-aware placement of the split layout's segments.
// k_vcache's compute lane ct of step s takes positions ct and CT + ct of the
// segment; every wave-instruction of the apply reads x[col] and y[row] with
// ds_read_b64 (bank pair (addr / 8) mod 32 per 32-lane half) and writes y[row]
// with ds_write_b64 (row mod 16 per 16-lane quarter), so a half whose 32
// entries repeat a column class (col mod 32) or a row class (row mod 32) is
// served in as many LDS cycles as the largest repeat.  In (row, column) order
// random columns cost ~3.5 cycles per half (3.64 conflict cycles
// per LDS instruction).  Here every 32-position group of a segment is filled
// with a maximum matching between column classes and row classes of the
// entries still unplaced (Kuhn's augmenting paths over 32 x 32 bitmasks), the
// rest of the group with the entries that add the fewest repeats, and each
// half of a group gets distinct row mod 16 where it can.  A segment's
// multi-entry row runs keep their consecutive positions (CONT / MORE) at its
// start, inside one wave.  Only the order of rows inside a segment changes --
// every row still has one run per segment in column order -- so every row's
// sum, and the result, is bit-identical to the (row, column) layout.
namespace {
struct BankPlacer {
  uint32_t CT;
  std::vector<uint32_t> code, out;  // scratch: the segment, slot -> source entry
  std::vector<uint64_t> vals;
  std::vector<uint32_t> pair_head, pair_next;  // per (cc, rc) pair: a list of single entries
  uint32_t cnt[32][32], adjbit[32], adjrank[32], cleft[32], rleft[32];
  int rorder[32], rank[32];  // row classes by singles at the segment's start (most first), and back
  std::vector<std::vector<uint32_t>> members;  // per group of 32 positions: its singles
  std::vector<std::array<uint8_t, 32>> gc, gr;  // per group: column / row class counts (runs included)
  explicit BankPlacer(uint32_t ct) : CT(ct), pair_head(1024) {}

  static int dfs(int c, const uint32_t* adj, int* match, uint32_t& visited) {
    for (uint32_t m = adj[c] & ~visited; m; m &= m - 1) {
      const int k = __builtin_ctz(m);
      visited |= 1u << k;
      if (match[k] < 0 || dfs(match[k], adj, match, visited)) {
        match[k] = c;
        return 1;
      }
    }
    return 0;
  }
  static int dfs64(int c, const uint64_t* adj, int* match, uint64_t& visited) {
    for (uint64_t m = adj[c] & ~visited; m; m &= m - 1) {
      const int k = __builtin_ctzll(m);
      visited |= 1ull << k;
      if (match[k] < 0 || dfs64(match[k], adj, match, visited)) {
        match[k] = c;
        return 1;
      }
    }
    return 0;
  }
  uint32_t take(uint32_t c, uint32_t r) {  // one single of pair (c, r)
    const uint32_t k = c * 32 + r, e = pair_head[k];
    pair_head[k] = pair_next[e];
    if (--cnt[c][r] == 0) {
      adjbit[c] &= ~(1u << r);
      adjrank[c] &= ~(1u << rank[r]);
    }
    cleft[c]--;
    rleft[r]--;
    return e;
  }

  // entries [s0, s1) of C / V (global arrays), rewritten in place; false: the
  // segment keeps its (row, column) order (its runs may then cross DPP rows)
  bool operator()(uint32_t* C, uint64_t* V, uint32_t s0, uint32_t s1) {
    const uint32_t n = s1 - s0;
    if (n < 2) return true;
    if (n > 2 * CT) return false;
    code.assign(C + s0, C + s1);
    vals.assign(V + s0, V + s1);
    out.assign(n, UINT32_MAX);
    auto cc = [&](uint32_t e) { return code[e] & 31u; };
    auto rc = [&](uint32_t e) { return (code[e] >> 16) & 31u; };
    // 1. multi-entry runs at the front, packed, none across a 16-position DPP
    // row (so none across a wave either)
    uint32_t p = 0;
    std::fill(pair_head.begin(), pair_head.end(), UINT32_MAX);
    pair_next.assign(n, UINT32_MAX);
    std::memset(cnt, 0, sizeof cnt);
    std::memset(adjbit, 0, sizeof adjbit);
    std::memset(cleft, 0, sizeof cleft);
    std::memset(rleft, 0, sizeof rleft);
    for (uint32_t e = 0; e < n;) {
      uint32_t f = e + 1;
      while (f < n && (code[f] & kVcCont)) ++f;
      const uint32_t len = f - e;
      if (len >= 2) {
        if (len > 16) return false;  // no DPP row holds it: keep the (row, column) order
        if ((p % 16) + len > 16) p = (p + 15) / 16 * 16;
        if (p + len > n) return false;  // cannot pack (tiny segment): keep the (row, column) order
        for (uint32_t q = 0; q < len; ++q) out[p + q] = e + q;
        p += len;
      } else {  // a single: into its (column class, row class) list
        const uint32_t c = cc(e), r = rc(e), k = c * 32 + r;
        pair_next[e] = pair_head[k];
        pair_head[k] = e;
        cnt[c][r]++;
        adjbit[c] |= 1u << r;
        cleft[c]++;
        rleft[r]++;
      }
      e = f;
    }
    for (int i = 0; i < 32; ++i) rorder[i] = i;
    std::sort(rorder, rorder + 32, [&](int x, int y) { return rleft[x] > rleft[y]; });
    for (int i = 0; i < 32; ++i) rank[rorder[i]] = i;
    for (int c = 0; c < 32; ++c) {
      adjrank[c] = 0;
      for (uint32_t bb = adjbit[c]; bb; bb &= bb - 1) adjrank[c] |= 1u << rank[__builtin_ctz(bb)];
    }
    // 2. groups of 32 positions: a maximum matching of column classes to row
    // classes, the classes with the most singles preferred on both sides,
    // then the entries adding the fewest repeats
    const uint32_t ng = (n + 31) / 32;
    members.assign(ng, {});
    gc.assign(ng, {});
    gr.assign(ng, {});
    for (uint32_t g = 0; g < ng; ++g) {
      const uint32_t g0 = g * 32, g1 = std::min(n, g0 + 32);
      uint32_t used_c = 0, used_r = 0, nfree = 0;
      for (uint32_t q = g0; q < g1; ++q) {
        if (out[q] == UINT32_MAX) {
          ++nfree;
          continue;
        }
        const uint32_t e = out[q];
        used_c |= 1u << cc(e);
        gc[g][cc(e)]++;
        if (!(code[e] & kVcCont)) {
          used_r |= 1u << rc(e);
          gr[g][rc(e)]++;
        }
      }
      if (!nfree) continue;
      // each class may appear cap = ceil(singles left / groups left) times (1 or
      // 2 copies in the matching), so the classes with more singles than
      // groups spread their repeats over every group instead of crowding the last
      const uint32_t gl = ng - g;
      int corder[32];
      for (int i = 0; i < 32; ++i) corder[i] = i;
      std::sort(corder, corder + 32, [&](int x, int y) { return cleft[x] > cleft[y]; });
      auto cap = [&](uint32_t left, uint32_t used) {
        const uint32_t c = std::min<uint32_t>(2, (left + gl - 1) / gl);
        return c > used ? c - used : 0u;
      };
      // row copy k of rank i is bit i + 32 k; column copies are nodes c + 32 k
      uint64_t rmask = 0;
      for (int i = 0; i < 32; ++i) {
        const uint32_t r = (uint32_t)rorder[i], cr = cap(rleft[r], gr[g][r]);
        if (cr >= 1) rmask |= 1ull << i;
        if (cr >= 2) rmask |= 1ull << (i + 32);
      }
      uint64_t adj[64];
      int cnodes[64], ncn = 0;
      for (int k = 0; k < 2; ++k)
        for (int i = 0; i < 32; ++i) {
          const int c = corder[i];
          adj[c + 32 * k] = 0;
          if (cap(cleft[c], gc[g][c]) <= (uint32_t)k) continue;
          adj[c + 32 * k] = ((uint64_t)adjrank[c] | (uint64_t)adjrank[c] << 32) & rmask;
          cnodes[ncn++] = c + 32 * k;
        }
      // augment in three phases: no repeat, then the column repeats the
      // schedule asks for, then the row repeats
      int match[64];
      std::fill(match, match + 64, -1);
      uint32_t size = 0;
      bool matched[64] = {false};
      for (int phase = 0; phase < 3 && size < nfree; ++phase) {
        const uint64_t allow = phase < 2 ? 0xFFFFFFFFull : ~0ull;
        uint64_t adjp[64];
        for (int i = 0; i < ncn; ++i) adjp[cnodes[i]] = adj[cnodes[i]] & allow;
        uint64_t taken_rows = 0;
        for (int k = 0; k < 64; ++k)
          if (match[k] >= 0) taken_rows |= 1ull << k;
        for (int i = 0; i < ncn && size < nfree; ++i) {  // greedy first: most nodes match directly
          const int cn = cnodes[i];
          if (matched[cn] || (phase == 0 && cn >= 32)) continue;
          const uint64_t m = adjp[cn] & ~taken_rows;
          if (!m) continue;
          const int k = __builtin_ctzll(m);
          match[k] = cn;
          taken_rows |= 1ull << k;
          matched[cn] = true;
          ++size;
        }
        for (int i = 0; i < ncn && size < nfree; ++i) {  // then augmenting paths
          const int cn = cnodes[i];
          if (matched[cn] || (phase == 0 && cn >= 32)) continue;
          uint64_t vis = 0;
          if (dfs64(cn, adjp, match, vis)) {
            matched[cn] = true;
            ++size;
          }
        }
      }
      auto add = [&](uint32_t c, uint32_t r) {
        members[g].push_back(take(c, r));
        gc[g][c]++;
        gr[g][r]++;
        used_c |= 1u << c;
        used_r |= 1u << r;
      };
      for (int k = 0; k < 64; ++k)
        if (match[k] >= 0) {
          const uint32_t c = (uint32_t)(match[k] & 31), r = (uint32_t)rorder[k & 31];
          if (cnt[c][r]) add(c, r);  // (a pair matched twice with one single left: the fill below)
        }
      while (members[g].size() < nfree) {
        int bc = -1, br = -1, best = 3;
        for (int i = 0; i < 32 && best; ++i) {
          const int c = corder[i];
          for (uint32_t bb = adjbit[c]; bb && best; bb &= bb - 1) {
            const int r = __builtin_ctz(bb);
            const int sc = (int)(used_c >> c & 1) + (int)(used_r >> r & 1);
            if (sc < best) {
              best = sc;
              bc = c;
              br = r;
            }
          }
        }
        if (bc < 0) return false;  // (the free slots equal the singles left: not reached) keep the old order
        add((uint32_t)bc, (uint32_t)br);
      }
    }
    // 3. inside each group: distinct row mod 16 per half where possible
    for (uint32_t g = 0; g < ng; ++g) {
      const uint32_t g0 = g * 32, g1 = std::min(n, g0 + 32);
      uint32_t used_h[2] = {0, 0}, hfree[2] = {0, 0}, placed[2] = {0, 0};
      for (uint32_t q = g0; q < g1; ++q) {
        if (out[q] == UINT32_MAX) {
          hfree[(q - g0) / 16]++;
        } else if (!(code[out[q]] & kVcCont)) {
          used_h[(q - g0) / 16] |= 1u << (rc(out[q]) & 15);
        }
      }
      uint32_t half[2][32], rest[32], nh[2] = {0, 0}, nrest = 0;
      for (uint32_t e : members[g]) {
        const uint32_t bit = 1u << (rc(e) & 15);
        int hh = -1;
        for (int x = 0; x < 2 && hh < 0; ++x)
          if (placed[x] < hfree[x] && !(used_h[x] & bit)) hh = x;
        if (hh < 0) {
          rest[nrest++] = e;
          continue;
        }
        used_h[hh] |= bit;
        half[hh][nh[hh]++] = e;
        placed[hh]++;
      }
      for (uint32_t i = 0; i < nrest; ++i) {
        const int hh = placed[0] < hfree[0] ? 0 : 1;
        half[hh][nh[hh]++] = rest[i];
        placed[hh]++;
      }
      size_t i0 = 0, i1 = 0;
      for (uint32_t q = g0; q < g1; ++q)
        if (out[q] == UINT32_MAX) out[q] = (q - g0) < 16 ? half[0][i0++] : half[1][i1++];
    }
    for (uint32_t q = 0; q < n; ++q) {
      C[s0 + q] = code[out[q]];
      V[s0 + q] = vals[out[q]];
    }
    return true;
  }
};
}  // namespace

void place_segments_banked(VcacheLayout& L, uint32_t CT) {
  const uint32_t units = L.nblocks * (uint32_t)L.geom.split, npad = L.npad;
  const unsigned nt = std::max(1u, std::min(plan_threads(), units));
  std::atomic<bool> all{true};
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    BankPlacer place(CT);
    bool ok = true;
    for (uint64_t t = t0; t < t1; ++t)
      for (uint32_t u = (uint32_t)t; u < units; u += nt) {
        const uint32_t* sg = &L.seg[(size_t)u * (npad + 1)];
        for (uint32_t i = 0; i < npad; ++i) ok = place(L.code.data(), L.vals.data(), sg[i], sg[i + 1]) && ok;
      }
    if (!ok) all = false;
  });
  // a segment left in (row, column) order may hold a run across a DPP row
  L.row_runs = all;
}

// k_vflow's layout (csrc/vflow.hip): build_vcache's segments over kVfGeom,
// each segment regrouped by owning compute wave (vf_wave_of of the row,
// stable: every row keeps its one run and its column order), each group then
// placed for LDS banks with its runs inside 16-lane DPP rows (BankPlacer, the
// group is the wave's two 64-lane slots; where it cannot pack the runs, the
// group keeps (row, column) order and only a run across a slot is refused).  Group (u, w, i) -- unit u, wave w,
// step i -- holds entries [wbeg, wend).  Only the order of rows inside a step
// changes, so every row's sum is the same sequence as in (row, column) order.
bool build_vflow(const HostCSR& a, VflowLayout& out) {
  const VcGeom& g = kVfGeom;
  if (!vcache_eligible(a, g) || vcache_max_run(a, (uint32_t)g.panel) > 16) return false;
  VcacheLayout& L = out.L;
  build_vcache(a, g, L);
  const uint32_t units = L.nblocks * (uint32_t)g.split, npad = L.npad, W = (uint32_t)kVfWaves;
  out.wbeg.resize((size_t)units * W * npad);
  out.wend.resize((size_t)units * W * npad);
  const unsigned nt = std::max(1u, std::min(plan_threads(), units));
  std::atomic<bool> ok{true};
  std::vector<uint32_t> tmax(nt, 0);
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    BankPlacer place(64);
    std::vector<uint32_t> code;
    std::vector<uint64_t> vals;
    for (uint64_t t = t0; t < t1; ++t)
      for (uint32_t u = (uint32_t)t; u < units && ok; u += nt) {
        const uint32_t* sg = &L.seg[(size_t)u * (npad + 1)];
        for (uint32_t i = 0; i < npad; ++i) {
          const uint32_t s0 = sg[i], s1 = sg[i + 1];
          uint32_t cnt[kVfWaves + 1] = {0};
          for (uint32_t e = s0; e < s1; ++e) cnt[vf_wave_of((L.code[e] >> 16) & 0x3FFFu) + 1]++;
          for (uint32_t w = 0; w < W; ++w) {
            tmax[t] = std::max(tmax[t], cnt[w + 1]);
            if (cnt[w + 1] > kVfGroupMax) ok = false;
            cnt[w + 1] += cnt[w];
          }
          code.assign(L.code.begin() + s0, L.code.begin() + s1);
          vals.assign(L.vals.begin() + s0, L.vals.begin() + s1);
          uint32_t cur[kVfWaves];
          for (uint32_t w = 0; w < W; ++w) {
            cur[w] = s0 + cnt[w];
            out.wbeg[((size_t)u * W + w) * npad + i] = s0 + cnt[w];
            out.wend[((size_t)u * W + w) * npad + i] = s0 + cnt[w + 1];
          }
          for (uint32_t q = 0; q < s1 - s0; ++q) {
            const uint32_t d = cur[vf_wave_of((code[q] >> 16) & 0x3FFFu)]++;
            L.code[d] = code[q];
            L.vals[d] = vals[q];
          }
          for (uint32_t w = 0; w < W && ok; ++w) {
            const uint32_t b0 = s0 + cnt[w], b1 = s0 + cnt[w + 1];
            if (b1 - b0 > kVfGroupMax) break;
            if (place(L.code.data(), L.vals.data(), b0, b1)) continue;
            // kept in (row, column) order (too few singles to pad the runs into 16-lane rows): a run
            // may cross a DPP row -- the kernel takes such a continuation by shuffle -- but never a
            // 64-lane slot
            for (uint32_t e = b0; e < b1; ++e)
              if ((L.code[e] & kVcCont) && ((e - b0) % 64) == 0) ok = false;
          }
        }
      }
  });
  if (!ok) return false;
  // wave-major inside each unit: wave w's groups of all steps back to back, so a wave streams one
  // contiguous range and only the boundary lines between its consecutive steps are shared (by the
  // same wave, one step apart); step-major order split every step's entries into 14 groups whose
  // boundary lines two waves fetched (measured 203 us on C3)
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    std::vector<uint32_t> code;
    std::vector<uint64_t> vals;
    for (uint64_t t = t0; t < t1; ++t)
      for (uint32_t u = (uint32_t)t; u < units; u += nt) {
        const uint32_t u0 = L.seg[(size_t)u * (npad + 1)], u1 = L.seg[(size_t)u * (npad + 1) + npad];
        code.assign(L.code.begin() + u0, L.code.begin() + u1);
        vals.assign(L.vals.begin() + u0, L.vals.begin() + u1);
        uint32_t d = u0;
        for (uint32_t w = 0; w < W; ++w)
          for (uint32_t i = 0; i < npad; ++i) {
            const size_t gi = ((size_t)u * W + w) * npad + i;
            const uint32_t b0 = out.wbeg[gi], b1 = out.wend[gi];
            out.wbeg[gi] = d;
            for (uint32_t e = b0; e < b1; ++e, ++d) {
              L.code[d] = code[e - u0];
              L.vals[d] = vals[e - u0];
            }
            out.wend[gi] = d;
          }
      }
  });
  out.max_group = *std::max_element(tmax.begin(), tmax.end());
  L.row_runs = ok;
  return ok;
}

// The k_vquad form of the vcache layout: the same blocks,
// panels and segment offsets, entries of a segment placed for a kernel whose
// step gives lane ct of the CT compute lanes the positions ct and CT + ct
// (two entries per lane, EPT = 2), code = col_local | row_local << 12 | flags:
//  * a row with two entries in the segment takes both slots of one lane
//    (first: kVqLMore, second: kVcCont) while lanes with two slots last, so the
//    lane adds its pair without any cross-lane step;
//  * longer runs (and pairs past that) take consecutive positions inside one
//    slot row and one 64-lane wave (kVcMore / kVcCont as in build_vcache): the
//    kernel finishes them with wave shuffles, never across a wave;
//  * single entries fill the rest.
// Rows are independent inside a segment, so the order of rows is free (FAST,
// u64); every row's entries stay in column order.  Returns false when a
// segment exceeds 2 * CT entries or a run cannot be placed that way.
bool build_vcache_lanes(const HostCSR& a, const VcGeom& g, uint32_t CT, VcacheLayout& out) {
  if (g.colbits != 12 || CT % 64 || CT == 0) return false;
  build_vcache(a, g, out);  // geometry, segment offsets and (row, col) order
  const uint32_t S = (uint32_t)g.split, npad = out.npad;
  hvec<uint32_t> code(out.code.size());
  hvec<uint64_t> vals(out.vals.size());
  std::atomic<bool> ok{true};
  const uint32_t units = out.nblocks * S;
  // units are independent (disjoint segments): strided over the threads
  const unsigned nt = std::max(1u, std::min(plan_threads(), units));
  par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
    std::vector<int64_t> pos;  // position of each entry of the segment (-1 unplaced)
    std::vector<uint8_t> used;
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    std::vector<size_t> multi;
    for (uint64_t t = t0; t < t1; ++t)
      for (uint32_t u = (uint32_t)t; u < units && ok.load(std::memory_order_relaxed); u += nt) {
        const uint32_t* sg = &out.seg[(size_t)u * (npad + 1)];
        for (uint32_t i = 0; i < npad; ++i) {
          const uint32_t s0 = sg[i], s1 = sg[i + 1], n = s1 - s0;
          if (!n) continue;
          if (n > 2 * CT) {
            ok = false;
            return;
          }
          // runs of the segment: [start, len) in storage (row, col) order
          runs.clear();
          for (uint32_t e = s0; e < s1;) {
            uint32_t f = e + 1;
            while (f < s1 && (out.code[f] & kVcCont)) ++f;
            runs.emplace_back(e, f - e);
            e = f;
          }
          const uint32_t m = n > CT ? n - CT : 0;  // lanes with a second slot
          pos.assign(n, -1);
          used.assign(n, 0);
          auto put = [&](uint32_t e, uint32_t p, uint32_t flags) {
            pos[e - s0] = p;
            used[p] = 1;
            code[s0 + p] = (out.code[e] & ~(kVcCont | kVcMore)) | flags;
            vals[s0 + p] = out.vals[e];
          };
          // 1. pairs lane-local on lanes [0, m)
          uint32_t lane = 0;
          for (auto& r : runs)
            if (r.second == 2 && lane < m) {
              put(r.first, lane, kVqLMore);
              put(r.first + 1, CT + lane, kVcCont);
              ++lane;
              r.second = 0;  // placed
            }
          // 2. other multi-entry runs: consecutive positions inside one slot row
          // and one wave, from the first free position on
          auto fits = [&](uint32_t p, uint32_t len) {
            if (p + len > n) return false;
            const uint32_t j = p / CT, c = p % CT;
            if ((p + len - 1) / CT != j || c / 64 != (c + len - 1) / 64) return false;
            for (uint32_t k = 0; k < len; ++k)
              if (used[p + k]) return false;
            return true;
          };
          // first fit, longest runs first (a run keeps its own entries in order)
          multi.clear();
          for (size_t k = 0; k < runs.size(); ++k)
            if (runs[k].second >= 2) multi.push_back(k);
          std::stable_sort(multi.begin(), multi.end(),
                           [&](size_t v, size_t w) { return runs[v].second > runs[w].second; });
          // a cursor at the first free position: every placement fills positions, so it
          // never moves back, and a run's search starts there (the scan from 0
          // made segments with many short runs quadratic)
          uint32_t cursor = 0;
          for (size_t k : multi) {
            auto& r = runs[k];
            while (cursor < n && used[cursor]) ++cursor;
            uint32_t p = cursor;
            while (p < n && !fits(p, r.second)) ++p;
            if (p >= n) {
              ok = false;
              return;
            }
            for (uint32_t q = 0; q < r.second; ++q)
              put(r.first + q, p + q, (q ? kVcCont : 0u) | (q + 1 < r.second ? kVcMore : 0u));
            r.second = 0;
          }
          // 3. single entries in order into the free positions
          uint32_t p = 0;
          for (auto& r : runs) {
            if (r.second != 1) continue;
            while (used[p]) ++p;
            put(r.first, p, 0u);
          }
        }
      }
  });
  if (!ok) return false;
  out.code.swap(code);
  out.vals.swap(vals);
  return true;
}

// SELL-C-sigma layout for k_sell (hipspmv_internal.h): within each window of
// kSellSigma rows the rows of at most kSellHub entries are ordered by length,
// longest first (ties by row id), and cut into slices of kSellRows; each
// row's entries keep their CSR order (ascending column = SoftwareSpMV's
// order), so the lane that owns a row adds them exactly as the reference does.
void build_sell(const HostCSR& a, SellLayout& out) {
  out = SellLayout{};
  auto len = [&](uint32_t r) { return a.rowptr[r + 1] - a.rowptr[r]; };
  const uint32_t nwin = (uint32_t)(((uint64_t)a.rows + kSellSigma - 1) / kSellSigma);
  // the windows are independent: sorted in parallel, laid out at offsets
  // from a serial prefix sum, filled in parallel -- the same bytes as a
  // serial build
  const unsigned nthr = std::max(1u, std::min(plan_threads(), nwin));
  auto parallel = [&](auto&& fn) {
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nthr; ++t)
      ts.emplace_back([&, t] {
        for (uint32_t w = t; w < nwin; w += nthr) fn(w);
      });
    for (auto& th : ts) th.join();
  };
  std::vector<std::vector<uint32_t>> order(nwin), whubs(nwin);
  parallel([&](uint32_t w) {
    const uint32_t w0 = w * kSellSigma, w1 = (uint32_t)std::min<uint64_t>((uint64_t)w0 + kSellSigma, a.rows);
    for (uint32_t r = w0; r < w1; ++r) (len(r) > kSellHub ? whubs[w] : order[w]).push_back(r);
    std::stable_sort(order[w].begin(), order[w].end(), [&](uint32_t p, uint32_t q) { return len(p) > len(q); });
  });
  std::vector<uint32_t> first_slice(nwin + 1, 0);
  for (uint32_t w = 0; w < nwin; ++w)
    first_slice[w + 1] = first_slice[w] + (uint32_t)((order[w].size() + kSellRows - 1) / kSellRows);
  const uint32_t nslices = first_slice[nwin];
  out.width.resize(nslices);
  out.off.resize((size_t)nslices + 1);
  out.off[0] = 0;
  for (uint32_t w = 0; w < nwin; ++w)
    for (uint32_t s = first_slice[w]; s < first_slice[w + 1]; ++s) {
      out.width[s] = len(order[w][(size_t)(s - first_slice[w]) * kSellRows]);  // longest first
      out.off[s + 1] = out.off[s] + (uint64_t)out.width[s] * kSellRows;
    }
  out.col.resize(out.off[nslices]);
  out.vals.resize(out.off[nslices]);
  out.row.resize((size_t)nslices * kSellRows);
  out.len.resize((size_t)nslices * kSellRows);
  parallel([&](uint32_t w) {
    const auto& ord = order[w];
    {  // the window's slices start as padding: column 0, value 0, no row
      const uint32_t s0 = first_slice[w], s1 = first_slice[w + 1];
      std::fill(out.col.begin() + out.off[s0], out.col.begin() + out.off[s1], 0u);
      std::fill(out.vals.begin() + out.off[s0], out.vals.begin() + out.off[s1], 0u);
      std::fill(out.row.begin() + (size_t)s0 * kSellRows, out.row.begin() + (size_t)s1 * kSellRows, kSellNoRow);
      std::fill(out.len.begin() + (size_t)s0 * kSellRows, out.len.begin() + (size_t)s1 * kSellRows, 0u);
    }
    for (size_t i = 0; i < ord.size(); ++i) {
      const uint32_t s = first_slice[w] + (uint32_t)(i / kSellRows), q = (uint32_t)(i % kSellRows);
      const uint32_t j = q / 64, l = q % 64;
      const uint32_t r = ord[i], e0 = a.rowptr[r], n = len(r);
      out.row[(size_t)s * kSellRows + q] = r;
      out.len[(size_t)s * kSellRows + q] = n;
      for (uint32_t k = 0; k < n; ++k) {
        const uint64_t d = out.off[s] + ((uint64_t)k * 4 + j) * 64 + l;
        out.col[d] = a.colind[e0 + k];
        out.vals[d] = a.vals[e0 + k];
      }
    }
  });
  std::vector<uint32_t> hubs;
  for (auto& v : whubs) hubs.insert(hubs.end(), v.begin(), v.end());
  std::stable_sort(hubs.begin(), hubs.end(), [&](uint32_t p, uint32_t q) {
    return a.rowptr[p + 1] - a.rowptr[p] > a.rowptr[q + 1] - a.rowptr[q];
  });
  uint64_t hub_nnz = 0;
  for (uint32_t r : hubs) hub_nnz += a.rowptr[r + 1] - a.rowptr[r];
  out.padding = out.off.back() - (a.nnz - hub_nnz);
  for (uint32_t r : hubs) {  // FAST pieces: near-equal cuts of at most kSellPiece entries
    const uint32_t n = a.rowptr[r + 1] - a.rowptr[r];
    const uint32_t np = (n + kSellPiece - 1) / kSellPiece;
    const uint32_t ticket = np > 1 ? out.ntickets++ : 0u;
    for (uint32_t p = 0; p < np; ++p) {
      const uint32_t b = (uint32_t)((uint64_t)n * p / np), e = (uint32_t)((uint64_t)n * (p + 1) / np);
      const uint32_t rec[kSellPieceWords] = {r, b, e - b, p, np, ticket, 0u, 0u};
      out.pieces.insert(out.pieces.end(), rec, rec + kSellPieceWords);
    }
  }
  out.npieces = (uint32_t)(out.pieces.size() / kSellPieceWords);
  out.niso = 0;  // hubs[0, niso): long enough for a workgroup of their own (ORDERED, k_sell_iso)
  while (out.niso < hubs.size() && a.rowptr[hubs[out.niso] + 1] - a.rowptr[hubs[out.niso]] >= kSellIso) ++out.niso;
  out.hubs = std::move(hubs);
  out.nhubs = (uint32_t)out.hubs.size();
  out.nslices = nslices;
}

// Column-windowed segment matrix (k_wreduce / wcsr, hipspmv_internal.h):
// segment (w, r) holds row r's entries with column in window w, in their CSR
// (ascending column) order; segments are numbered window-major, rows ascending
// within a window, so a kernel walking them in order gathers from one window
// of x at a time.  For each row, its segment ids in window order.
uint64_t windowed_segments(const HostCSR& a, uint32_t log2w) {
  std::vector<uint64_t> n(plan_threads() + 1, 0);
  par_rows(a.rowptr.data(), a.rows, [&](unsigned t, uint32_t r0, uint32_t r1) {
    uint64_t k = 0;
    for (uint32_t r = r0; r < r1; ++r) {
      uint32_t prev = UINT32_MAX;
      for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e) {
        const uint32_t w = a.colind[e] >> log2w;
        k += w != prev;
        prev = w;
      }
    }
    n[t] = k;
  });
  uint64_t s = 0;
  for (uint64_t k : n) s += k;
  return s;
}

// The row partition of a multi-device handle (hipspmv_partition_rows; VERDICT
// r04 item 3): contiguous blocks of about equal cost, where a row costs
//   entries + segments + 1
// in units of one entry's time, with its segments counted exactly as
// build_windowed cuts them for the wcsr kernel: one per run of the row inside a
// 2^kWcLog2Window-column window, runs longer than kCvGroupNnz cut into pieces.
// The unit weights are wcsr's measured costs rounded (per entry, per segment
// partial, per row of output: 7.08 / 6.77 / 7.51 us per million on an MI355X,
// profiles/r04/logs/bench_c5_w20.log) -- constants of the kernel, not of a
// matrix.  On rows of equal shape (the stripe matrices, whose kernels stream
// entries) the cost is proportional to the entries, so the partition is the
// entry-balanced one; on R-MAT it charges the short-row blocks their segments
// and rows (C5: the nnz-balanced cut spread the shard times 1.66x).
// Interior bounds snap to the nearer multiple of HIPSPMV_SHARD_ALIGN.
void partition_rows_cost(const uint32_t* rowptr, const uint32_t* colind, uint32_t rows, uint32_t parts,
                         uint32_t* bounds) {
  std::vector<double> cum((size_t)rows + 1, 0.0);
  par_rows(rowptr, rows, [&](unsigned, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1; ++r) {
      uint64_t seg = 0;
      for (uint32_t e = rowptr[r]; e < rowptr[r + 1];) {
        const uint32_t w = colind[e] >> kWcLog2Window;
        uint32_t f = e + 1;
        while (f < rowptr[r + 1] && (colind[f] >> kWcLog2Window) == w) ++f;
        seg += (f - e + kCvGroupNnz - 1) / kCvGroupNnz;
        e = f;
      }
      cum[(size_t)r + 1] = (double)(rowptr[r + 1] - rowptr[r]) + (double)seg + 1.0;
    }
  });
  for (uint32_t r = 0; r < rows; ++r) cum[(size_t)r + 1] += cum[r];
  const uint32_t A = HIPSPMV_SHARD_ALIGN;
  bounds[0] = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    const double target = cum[rows] * p / parts;
    uint32_t r = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
    r = std::min(r, rows);
    const uint32_t lo = r / A * A;
    const uint32_t snap = std::min(rows, r - lo <= A / 2 ? lo : lo + A);
    bounds[p] = std::max(snap, bounds[p - 1]);
  }
  bounds[parts] = rows;
}

// In parallel over entry-balanced row ranges (thread t: rows [rb[t], rb[t+1])):
// a window's segments are numbered by rows ascending, so thread t's first
// segment of window w follows every earlier thread's segments of w.
void build_windowed(const HostCSR& a, uint32_t log2w, WinLayout& out, uint32_t cap, bool by_line) {
  out = WinLayout{};
  out.log2w = log2w;
  const uint32_t nwin = (uint32_t)(((uint64_t)a.cols + (1ull << log2w) - 1) >> log2w);
  // segment order: window-major, then (by_line) the 128-byte x line of the
  // segment's first column, then row -- one counting sort over the buckets
  // (lines, or windows); a window's buckets are contiguous either way
  const uint32_t bsh = by_line && log2w >= 4 ? 4 : log2w;
  const uint32_t nbk = (uint32_t)(((uint64_t)a.cols + (1ull << bsh) - 1) >> bsh);
  const unsigned nt = std::max(1u, std::min(plan_threads(), std::max(1u, a.rows / 64)));
  const std::vector<uint32_t> rb = row_chunks(a.rowptr.data(), a.rows, nt);
  auto each_thread = [&](auto&& fn) {
    par_chunks(nt, nt, [&](unsigned, uint64_t t0, uint64_t t1) {
      for (uint64_t t = t0; t < t1; ++t) fn((unsigned)t, rb[t], rb[t + 1]);
    });
  };
  // pass 1: segments per row and per (thread, bucket)
  std::vector<std::vector<uint32_t>> wcnt(nt, std::vector<uint32_t>(nbk, 0));
  out.rowseg.resize((size_t)a.rows + 1);
  each_thread([&](unsigned t, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1; ++r) {
      uint32_t prev = UINT32_MAX, n = 0, run = 0;
      for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e, ++run) {
        const uint32_t w = a.colind[e] >> log2w;
        if (w != prev || run == cap) {  // a new window, or the segment is full
          wcnt[t][a.colind[e] >> bsh]++;
          ++n;
          prev = w;
          run = 0;
        }
      }
      out.rowseg[r + 1] = n;
    }
  });
  out.rowseg[0] = 0;
  for (uint32_t r = 0; r < a.rows; ++r) out.rowseg[r + 1] += out.rowseg[r];
  std::vector<uint64_t> bstart((size_t)nbk + 1, 0);
  std::vector<std::vector<uint32_t>>& cursor = wcnt;  // counts -> cursors in place
  for (uint32_t k = 0; k < nbk; ++k) {
    uint64_t c = bstart[k];
    for (unsigned t = 0; t < nt; ++t) {
      const uint32_t n = wcnt[t][k];
      cursor[t][k] = (uint32_t)c;
      c += n;
    }
    bstart[k + 1] = c;
  }
  std::vector<uint64_t> wstart((size_t)nwin + 1, 0);
  for (uint32_t w = 0; w <= nwin; ++w)
    wstart[w] = bstart[std::min<uint64_t>((uint64_t)w << (log2w - bsh), nbk)];
  out.nseg = (uint32_t)wstart[nwin];
  out.winseg.assign(wstart.begin(), wstart.end());
  // pass 2: each segment's id (rows ascend, so ids ascend within a window) and length
  hvec<uint32_t> len(out.nseg);
  out.segidx.resize(out.nseg);
  each_thread([&](unsigned t, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1; ++r) {
      uint32_t prev = UINT32_MAX, k = out.rowseg[r], run = 0;
      for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e, ++run) {
        const uint32_t w = a.colind[e] >> log2w;
        if (w != prev || run == cap) {
          out.segidx[k] = cursor[t][a.colind[e] >> bsh]++;
          len[out.segidx[k]] = 0;
          ++k;
          prev = w;
          run = 0;
        }
        len[out.segidx[k - 1]]++;
      }
    }
  });
  HostCSR& g = out.seg;
  g.rows = out.nseg;
  g.cols = a.cols;
  g.nnz = a.nnz;
  g.rowptr.resize((size_t)out.nseg + 1);
  {  // rowptr = exclusive prefix of len, in two parallel passes over chunks
    const unsigned nc = std::max(1u, std::min(plan_threads(), std::max(1u, out.nseg / 4096)));
    std::vector<uint64_t> csum(nc + 1, 0);
    std::vector<uint32_t> cmax(nc, 0);
    par_chunks(out.nseg, nc, [&](unsigned c, uint64_t lo, uint64_t hi) {
      uint64_t s = 0;
      uint32_t m = 0;
      for (uint64_t i = lo; i < hi; ++i) {
        s += len[i];
        m = std::max(m, len[i]);
      }
      csum[c + 1] = s;
      cmax[c] = m;
    });
    for (unsigned c = 0; c < nc; ++c) csum[c + 1] += csum[c];
    par_chunks(out.nseg, nc, [&](unsigned c, uint64_t lo, uint64_t hi) {
      uint64_t s = csum[c];
      for (uint64_t i = lo; i < hi; ++i) {
        g.rowptr[i] = (uint32_t)s;
        s += len[i];
      }
    });
    g.rowptr[out.nseg] = a.nnz;
    out.max_seg = *std::max_element(cmax.begin(), cmax.end());
  }
  // pass 3: copy each row's entries into its segments
  g.colind.resize(a.nnz);
  g.vals.resize(a.nnz);
  each_thread([&](unsigned, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1; ++r) {
      uint32_t prev = UINT32_MAX, k = out.rowseg[r], d = 0, run = 0;
      for (uint32_t e = a.rowptr[r]; e < a.rowptr[r + 1]; ++e, ++run) {
        const uint32_t w = a.colind[e] >> log2w;
        if (w != prev || run == cap) {
          d = g.rowptr[out.segidx[k++]];
          prev = w;
          run = 0;
        }
        g.colind[d] = a.colind[e];
        g.vals[d] = a.vals[e];
        ++d;
      }
    }
  });
}

// The hot-column form (hipspmv_internal.h): one window per thread; a dense
// counter and slot map of the window's 2^log2w columns, the K most frequent
// columns by (count descending, column ascending), their slots in column
// order (the segment pass stages them in LDS with one gather per slot, so
// neighbouring slots share x lines).
bool mark_hot_columns(WinLayout& L, uint32_t K, std::vector<uint32_t>& hot) {
  HostCSR& g = L.seg;
  if ((uint64_t)g.cols > kWcHotFlag || K == 0) return false;
  const uint32_t nwin = (uint32_t)L.winseg.size() - 1, W = 1u << L.log2w;
  hot.assign((size_t)nwin * K, 0u);
  const unsigned nt = std::max(1u, std::min(plan_threads(), nwin));
  par_chunks(nwin, nt, [&](unsigned, uint64_t w0, uint64_t w1) {
    std::vector<uint32_t> cnt(W), slot(W);
    std::vector<uint64_t> cand;
    for (uint64_t w = w0; w < w1; ++w) {
      const uint64_t e0 = g.rowptr[L.winseg[w]], e1 = g.rowptr[L.winseg[w + 1]];
      if (e0 == e1) continue;
      const uint32_t c0 = (uint32_t)(w << L.log2w);
      std::fill(cnt.begin(), cnt.end(), 0u);
      for (uint64_t e = e0; e < e1; ++e) cnt[g.colind[e] - c0]++;
      cand.clear();
      for (uint32_t c = 0; c < W; ++c)  // key: count descending, then column ascending
        if (cnt[c]) cand.push_back((uint64_t)(UINT32_MAX - cnt[c]) << 32 | c);
      const size_t k = std::min<size_t>(K, cand.size());
      std::nth_element(cand.begin(), cand.begin() + (k ? k - 1 : 0), cand.end());
      std::vector<uint32_t> cols(k);
      for (size_t i = 0; i < k; ++i) cols[i] = (uint32_t)cand[i];
      std::sort(cols.begin(), cols.end());
      std::fill(slot.begin(), slot.end(), UINT32_MAX);
      uint32_t* hw = hot.data() + (size_t)w * K;
      for (size_t i = 0; i < k; ++i) {
        slot[cols[i]] = (uint32_t)i;
        hw[i] = c0 + cols[i];
      }
      for (size_t i = k; i < K; ++i) hw[i] = c0;  // padding: never referenced
      for (uint64_t e = e0; e < e1; ++e) {
        const uint32_t sl = slot[g.colind[e] - c0];
        if (sl != UINT32_MAX) g.colind[e] = kWcHotFlag | sl;
      }
    }
  });
  return true;
}

// Greedy row groups: consecutive rows while the group stays within
// kCvGroupNnz nonzeros and kCvGroupRows rows; a longer row is a group alone.
// No group crosses a multiple of HIPSPMV_SHARD_ALIGN rows, so the groups of a
// shard that starts at such a row are exactly the unpartitioned matrix's
// groups there, and csr_vector's reduction order -- and so its FAST-mode
// bits -- does not depend on the partition.
void build_xmask(const VcacheLayout& L, uint32_t WL, std::vector<uint64_t>& out) {
  const uint32_t units = L.nblocks * (uint32_t)L.geom.split, P = L.npanels, stride = L.npad + 1;
  const uint32_t cmask = (1u << L.geom.colbits) - 1u, lines_per_j = 8 * WL;
  out.assign((size_t)units * P * WL, 0ull);
  auto unit = [&](uint64_t u) {
    const uint32_t* sp = L.seg.data() + (size_t)u * stride;
    for (uint32_t s = 0; s < P && s < stride - 1; ++s) {
      uint64_t* w = out.data() + ((size_t)u * P + s) * WL;
      for (uint32_t e = sp[s]; e < sp[s + 1]; ++e) {
        // lines past 64 bits of a wave's word have no bit: the kernel applies the mask only where
        // every line has one (k_vcache XMASK: NJ * 8 <= 64)
        const uint32_t line = (L.code[e] & cmask) >> 4, j = line / lines_per_j, r = line % lines_per_j;
        if (j < 8) w[r / 8] |= 1ull << (j * 8 + r % 8);
      }
    }
  };
  par_chunks(units, plan_threads(), [&](unsigned, uint64_t lo, uint64_t hi) {
    for (uint64_t u = lo; u < hi; ++u) unit(u);
  });
}

void build_row_groups(const uint32_t* rowptr, uint32_t rows, std::vector<uint32_t>& groups) {
  static_assert(kCvGroupRows <= HIPSPMV_SHARD_ALIGN && HIPSPMV_SHARD_ALIGN % kCvGroupRows == 0,
                "a group fits an aligned window");
  groups.clear();
  uint32_t r = 0;
  while (r < rows) {
    groups.push_back(r);
    const uint32_t start = rowptr[r];
    uint32_t n = 0;
    while (r < rows && n < (uint32_t)kCvGroupRows && rowptr[r + 1] - start <= (uint32_t)kCvGroupNnz &&
           (n == 0 || r % HIPSPMV_SHARD_ALIGN != 0)) {
      ++r;
      ++n;
    }
    if (n == 0) ++r;  // a long row: its own group
  }
  groups.push_back(rows);
}
void build_row_groups(const HostCSR& a, std::vector<uint32_t>& groups) {
  build_row_groups(a.rowptr.data(), a.rows, groups);
}

}  // namespace hipspmv
