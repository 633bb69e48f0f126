#include "csr2csc.h"

#include <cstddef>
#include <vector>

namespace {
// Count entries per output column, exclusive-scan into column starts, then
// place row by row with a per-column cursor: entries of a column come out in
// ascending row order (stable), which the ordered SpMV modes rely on.
template <typename I, typename V>
void transpose(I n, I m, I nz, const V* a, const I* col_idx, const I* row_start, V* csc_a, I* row_idx,
               I* col_start) {
  std::vector<I> cursor((size_t)m + 1, 0);
  for (I i = 0; i < nz; ++i) cursor[col_idx[i] + 1]++;
  for (I j = 0; j < m; ++j) cursor[j + 1] += cursor[j];
  for (I j = 0; j <= m; ++j) col_start[j] = cursor[j];
  for (I r = 0; r < n; ++r) {
    for (I e = row_start[r]; e < row_start[r + 1]; ++e) {
      const I dst = cursor[col_idx[e]]++;
      row_idx[dst] = r;
      if (a) csc_a[dst] = a[e];
    }
  }
}
}  // namespace

void csr2csc(int n, int m, int nz, double* a, int* col_idx, int* row_start, double* csc_a, int* row_idx,
             int* col_start) {
  transpose<int, double>(n, m, nz, a, col_idx, row_start, csc_a, row_idx, col_start);
}

void csr2csc(uint32_t n, uint32_t m, uint32_t nz, const uint64_t* a, const uint32_t* col_idx,
             const uint32_t* row_start, uint64_t* csc_a, uint32_t* row_idx, uint32_t* col_start) {
  transpose<uint32_t, uint64_t>(n, m, nz, a, col_idx, row_start, csc_a, row_idx, col_start);
}
