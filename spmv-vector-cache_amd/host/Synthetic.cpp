#include "Synthetic.h"

#include "hipspmv.h"

#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <thread>

uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double uniform11(uint64_t z) { return (double)(z >> 11) * 0x1.0p-52 - 1.0; }

unsigned hostThreads() {
  for (const char* var : {"SPMV_THREADS", "OMP_NUM_THREADS"}) {
    if (const char* s = std::getenv(var)) {
      const long v = std::strtol(s, nullptr, 10);
      if (v > 0) return (unsigned)std::min<long>(v, 256);
    }
  }
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Runs f(t, begin, end) on contiguous chunks [begin, end) of [0, n), chunk t
// before chunk t+1, one std::thread per chunk (no OpenMP runtime: the host
// library is loaded into processes that carry their own).
template <typename F>
static void parallelChunks(uint64_t n, unsigned nt, F f) {
  nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nt, n / 65536 + 1));
  if (nt == 1) {
    f(0u, (uint64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < nt; ++t) pool.emplace_back(f, t, n * t / nt, n * (t + 1) / nt);
  for (auto& th : pool) th.join();
}

void genStripeCSR(uint64_t row0, uint32_t nrows, uint32_t cols, uint32_t k, uint64_t seedCol, uint64_t seedVal,
                  uint32_t* rowptr, uint32_t* colind, double* vals) {
  std::vector<uint32_t> lo(k + 1);
  for (uint32_t j = 0; j <= k; ++j) lo[j] = (uint32_t)((uint64_t)j * cols / k);
  parallelChunks(nrows, hostThreads(), [&](unsigned, uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint64_t r = row0 + i;
      const uint64_t e0 = i * k;
      for (uint32_t j = 0; j < k; ++j) {
        const uint64_t g = r * k + j;
        const uint32_t w = lo[j + 1] - lo[j];
        colind[e0 + j] = lo[j] + (uint32_t)(splitmix64_at(seedCol, g) % w);
        vals[e0 + j] = uniform11(splitmix64_at(seedVal, g));
      }
    }
  });
  for (uint64_t i = 0; i <= nrows; ++i) rowptr[i] = (uint32_t)(i * k);
}

namespace {

struct RmatParams {
  uint32_t scale;
  uint64_t seed;
  double a, ab, abc;
};

// Edge i: one quadrant per level from u = (splitmix64_at(seed, i*scale+lvl)
// >> 11) * 2^-53 (Graph500 R-MAT).
inline void rmatEdge(const RmatParams& p, uint64_t i, uint64_t& r, uint64_t& c) {
  r = 0;
  c = 0;
  for (uint32_t lvl = 0; lvl < p.scale; ++lvl) {
    const double u = (double)(splitmix64_at(p.seed, i * p.scale + lvl) >> 11) * 0x1.0p-53;
    const uint64_t bit = 1ull << (p.scale - 1 - lvl);
    if (u < p.a) {
    } else if (u < p.ab) {
      c |= bit;
    } else if (u < p.abc) {
      r |= bit;
    } else {
      r |= bit;
      c |= bit;
    }
  }
}

}  // namespace

void genRmatRowCounts(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                      uint32_t* counts) {
  const uint64_t n = 1ull << scale, m = n * edgeFactor;
  const RmatParams p{scale, seed, a, a + b, a + b + c};
  std::fill(counts, counts + n, 0u);
  parallelChunks(m, hostThreads(), [&](unsigned, uint64_t b0, uint64_t e0) {
    for (uint64_t i = b0; i < e0; ++i) {
      uint64_t r, cc;
      rmatEdge(p, i, r, cc);
      __atomic_fetch_add(&counts[r], 1u, __ATOMIC_RELAXED);
    }
  });
}

uint64_t genRmatCSRRows(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                        uint32_t row0, uint32_t row1, std::vector<uint32_t>& rowptr, std::vector<uint32_t>& colind,
                        std::vector<double>& vals) {
  const uint64_t n = 1ull << scale, m = n * edgeFactor;
  row1 = (uint32_t)std::min<uint64_t>(row1, n);
  row0 = std::min(row0, row1);
  const uint32_t nr = row1 - row0;
  const RmatParams p{scale, seed, a, a + b, a + b + c};
  // 1. the edges of rows [row0, row1), per thread in edge order
  const unsigned nt = hostThreads();
  std::vector<std::vector<uint64_t>> tkey(nt);  // (row - row0) << 32 | col
  std::vector<std::vector<double>> tval(nt);
  parallelChunks(m, nt, [&](unsigned t, uint64_t b0, uint64_t e0) {
    for (uint64_t i = b0; i < e0; ++i) {
      uint64_t r, cc;
      rmatEdge(p, i, r, cc);
      if (r < row0 || r >= row1) continue;
      tkey[t].push_back(((r - row0) << 32) | cc);
      tval[t].push_back(uniform11(splitmix64_at(seed + 1, i)));
    }
  });
  // 2. stable counting sort by row (threads in chunk order = edge order)
  std::vector<uint64_t> start(nr + 1, 0);
  for (const auto& v : tkey)
    for (uint64_t k : v) start[(k >> 32) + 1]++;
  for (uint32_t r = 0; r < nr; ++r) start[r + 1] += start[r];
  const uint64_t me = start[nr];
  std::vector<uint32_t> col(me);
  std::vector<double> val(me);
  {
    std::vector<uint64_t> cur(start.begin(), start.end() - 1);
    for (unsigned t = 0; t < nt; ++t) {
      for (size_t j = 0; j < tkey[t].size(); ++j) {
        const uint64_t d = cur[tkey[t][j] >> 32]++;
        col[d] = (uint32_t)(tkey[t][j] & 0xFFFFFFFFu);
        val[d] = tval[t][j];
      }
      std::vector<uint64_t>().swap(tkey[t]);
      std::vector<double>().swap(tval[t]);
    }
  }
  // 3. per row: stable sort by column, sum duplicates in edge order
  std::vector<uint32_t> len(nr);
  parallelChunks(nr, nt, [&](unsigned, uint64_t b0, uint64_t e0) {
    std::vector<std::pair<uint32_t, double>> tmp;
    for (uint64_t r = b0; r < e0; ++r) {
      const uint64_t s = start[r], e = start[r + 1];
      tmp.clear();
      for (uint64_t j = s; j < e; ++j) tmp.emplace_back(col[j], val[j]);
      std::stable_sort(tmp.begin(), tmp.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
      uint64_t w = s;
      for (size_t j = 0; j < tmp.size(); ++j) {
        if (j && tmp[j].first == tmp[j - 1].first) {
          val[w - 1] += tmp[j].second;
          continue;
        }
        col[w] = tmp[j].first;
        val[w] = tmp[j].second;
        ++w;
      }
      len[r] = (uint32_t)(w - s);
    }
  });
  // 4. compact
  rowptr.assign((size_t)nr + 1, 0);
  for (uint32_t r = 0; r < nr; ++r) rowptr[r + 1] = rowptr[r] + len[r];
  const uint64_t nnz = rowptr[nr];
  colind.resize(nnz);
  vals.resize(nnz);
  for (uint32_t r = 0; r < nr; ++r) {
    std::copy(col.begin() + start[r], col.begin() + start[r] + len[r], colind.begin() + rowptr[r]);
    std::copy(val.begin() + start[r], val.begin() + start[r] + len[r], vals.begin() + rowptr[r]);
  }
  return nnz;
}

uint64_t genRmatCSR(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                    std::vector<uint32_t>& rowptr, std::vector<uint32_t>& colind, std::vector<double>& vals) {
  return genRmatCSRRows(scale, edgeFactor, seed, a, b, c, 0, (uint32_t)(1ull << scale), rowptr, colind, vals);
}

// Interior bounds move to the nearer multiple of HIPSPMV_SHARD_ALIGN rows
// (include/hipspmv.h): shards cut there compute every row with the
// unpartitioned matrix's bits in every kernel.
static uint32_t snapShardStart(uint32_t r, uint32_t rows) {
  const uint32_t a = HIPSPMV_SHARD_ALIGN, lo = std::min(r, rows) / a * a;
  return std::min(rows, std::min(r, rows) - lo <= a / 2 ? lo : lo + a);
}

void partitionRows(const uint32_t* rowptr, uint32_t rows, uint32_t parts, uint32_t* bounds) {
  const uint64_t nnz = rowptr[rows];
  bounds[0] = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    const uint64_t target = nnz * p / parts;
    // first row whose start reaches the target, snapped, never before the previous bound
    uint32_t r = (uint32_t)(std::lower_bound(rowptr, rowptr + rows + 1, (uint32_t)target) - rowptr);
    bounds[p] = std::max(snapShardStart(r, rows), bounds[p - 1]);
  }
  bounds[parts] = rows;
}

void partitionRowCounts(const uint32_t* counts, uint32_t rows, uint32_t parts, uint32_t* bounds) {
  uint64_t total = 0;
  for (uint32_t r = 0; r < rows; ++r) total += counts[r];
  bounds[0] = 0;
  uint64_t acc = 0;
  uint32_t r = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    const uint64_t target = total * p / parts;
    while (r < rows && acc < target) acc += counts[r++];
    bounds[p] = std::max(snapShardStart(r, rows), bounds[p - 1]);
  }
  bounds[parts] = rows;
}
