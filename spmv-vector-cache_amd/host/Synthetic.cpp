#include "Synthetic.h"

#include <algorithm>
#include <numeric>

uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double uniform11(uint64_t z) { return (double)(z >> 11) * 0x1.0p-52 - 1.0; }

void genStripeCSR(uint64_t row0, uint32_t nrows, uint32_t cols, uint32_t k, uint64_t seedCol, uint64_t seedVal,
                  uint32_t* rowptr, uint32_t* colind, double* vals) {
  std::vector<uint32_t> lo(k + 1);
  for (uint32_t j = 0; j <= k; ++j) lo[j] = (uint32_t)((uint64_t)j * cols / k);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)nrows; ++i) {
    const uint64_t r = row0 + (uint64_t)i;
    const uint64_t e0 = (uint64_t)i * k;
    for (uint32_t j = 0; j < k; ++j) {
      const uint64_t g = r * k + j;
      const uint32_t w = lo[j + 1] - lo[j];
      colind[e0 + j] = lo[j] + (uint32_t)(splitmix64_at(seedCol, g) % w);
      vals[e0 + j] = uniform11(splitmix64_at(seedVal, g));
    }
  }
  for (uint32_t i = 0; i <= nrows; ++i) rowptr[i] = i * k;
}

uint64_t genRmatCSR(uint32_t scale, uint32_t edgeFactor, uint64_t seed, double a, double b, double c,
                    std::vector<uint32_t>& rowptr, std::vector<uint32_t>& colind, std::vector<double>& vals) {
  const uint64_t n = 1ull << scale, m = n * edgeFactor;
  std::vector<uint64_t> key(m);  // (row << 32 | col)
  std::vector<double> v(m);
  const double ab = a + b, abc = a + b + c;
#pragma omp parallel for schedule(static)
  for (int64_t ii = 0; ii < (int64_t)m; ++ii) {
    const uint64_t i = (uint64_t)ii;
    uint64_t r = 0, cc = 0;
    for (uint32_t lvl = 0; lvl < scale; ++lvl) {
      const double u = (double)(splitmix64_at(seed, i * scale + lvl) >> 11) * 0x1.0p-53;
      const uint64_t bit = 1ull << (scale - 1 - lvl);
      if (u < a) {
      } else if (u < ab) {
        cc |= bit;
      } else if (u < abc) {
        r |= bit;
      } else {
        r |= bit;
        cc |= bit;
      }
    }
    key[i] = (r << 32) | cc;
    v[i] = uniform11(splitmix64_at(seed + 1, i));
  }
  std::vector<uint64_t> order(m);
  std::iota(order.begin(), order.end(), 0ull);
  std::stable_sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return key[x] < key[y]; });
  rowptr.assign(n + 1, 0);
  colind.clear();
  vals.clear();
  colind.reserve(m);
  vals.reserve(m);
  uint64_t prev = ~0ull;
  for (uint64_t i : order) {
    if (key[i] == prev) {
      vals.back() += v[i];
      continue;
    }
    prev = key[i];
    colind.push_back((uint32_t)(key[i] & 0xFFFFFFFFu));
    vals.push_back(v[i]);
    rowptr[(key[i] >> 32) + 1]++;
  }
  for (uint64_t r = 0; r < n; ++r) rowptr[r + 1] += rowptr[r];
  return colind.size();
}

void partitionRows(const uint32_t* rowptr, uint32_t rows, uint32_t parts, uint32_t* bounds) {
  const uint64_t nnz = rowptr[rows];
  bounds[0] = 0;
  for (uint32_t p = 1; p < parts; ++p) {
    const uint64_t target = nnz * p / parts;
    // first row whose start reaches the target, but never before the previous bound
    uint32_t r = (uint32_t)(std::lower_bound(rowptr, rowptr + rows + 1, (uint32_t)target) - rowptr);
    bounds[p] = std::max(std::min(r, rows), bounds[p - 1]);
  }
  bounds[parts] = rows;
}
