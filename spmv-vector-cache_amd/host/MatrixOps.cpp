#include "MatrixOps.h"

#include <algorithm>
#include <numeric>

namespace {
constexpr uint32_t kRowMask = 0x3FFFFFFFu;  // SparseMatrix.cpp:64,77 CMS bits

std::vector<uint32_t> rowLengths(const SparseMatrix* A) {
  std::vector<uint32_t> len(A->getRows(), 0);
  const SpMVIndex* inds = A->getInds();
  for (uint32_t e = 0; e < A->getNz(); ++e) len[inds[e] & kRowMask]++;
  return len;
}
}  // namespace

std::map<uint32_t, uint32_t> rowLenHistogram(const SparseMatrix* A) {
  const std::vector<uint32_t> len = rowLengths(A);
  std::map<uint32_t, uint32_t> h;
  // j = 1 .. cols-1 reads indptr[j] - indptr[j-1] = length of row j-1
  const uint32_t last = std::min<uint32_t>(A->getCols() ? A->getCols() - 1 : 0, A->getRows());
  for (uint32_t j = 1; j <= last; ++j) h[len[j - 1]]++;
  return h;
}

std::vector<uint32_t> longestRowFirstPermutation(const SparseMatrix* A) {
  const std::vector<uint32_t> len = rowLengths(A);
  std::vector<uint32_t> perm(A->getRows());
  std::iota(perm.begin(), perm.end(), 0u);
  std::sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
    return len[a] != len[b] ? len[a] > len[b] : a > b;
  });
  return perm;
}

SparseMatrix* permuteRows(const SparseMatrix* A, const std::vector<uint32_t>& perm) {
  const uint32_t rows = A->getRows(), cols = A->getCols(), nz = A->getNz();
  std::vector<uint32_t> inv(rows);
  for (uint32_t i = 0; i < rows; ++i) inv[perm[i]] = i;
  auto* colptr = new SpMVIndex[cols + 1];
  auto* inds = new SpMVIndex[nz];
  auto* data = new SpMVData[nz];
  const SpMVIndex* cp = A->getIndPtrs();
  const SpMVIndex* ri = A->getInds();
  const SpMVData* v = A->getNzData();
  std::vector<std::pair<uint32_t, SpMVData>> tmp;
  colptr[0] = 0;
  for (uint32_t c = 0; c < cols; ++c) {
    tmp.clear();
    for (uint32_t e = cp[c]; e < cp[c + 1]; ++e) tmp.emplace_back(inv[ri[e] & kRowMask], v[e]);
    std::stable_sort(tmp.begin(), tmp.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t k = 0; k < tmp.size(); ++k) {
      inds[cp[c] + k] = tmp[k].first;
      data[cp[c] + k] = tmp[k].second;
    }
    colptr[c + 1] = cp[c + 1];
  }
  SparseMatrix* P = SparseMatrix::fromArrays(rows, cols, nz, colptr, inds, data, A->getDataType(), true);
  return P;
}
