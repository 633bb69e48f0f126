// Offline matrix preparation of matrices/matrixutils.py that sits before the
// SpMV path: the row-length histogram (:116-126) and the longest-row-first
// row permutation (:140-158), on the reference's CSC SparseMatrix.
#ifndef SPMV_AMD_MATRIXOPS_H_
#define SPMV_AMD_MATRIXOPS_H_

#include <cstdint>
#include <map>
#include <vector>

#include "SparseMatrix.h"

// generateRowLenHistogram as written: its loop runs j = 1 .. shape[1]-1 over
// the CSR indptr, i.e. it counts the lengths of rows 0 .. cols-2 (the last row
// of a square matrix is left out); clamped to the rows that exist.  Row ids
// are read with the CMS bits masked.  {row length: number of rows}.
std::map<uint32_t, uint32_t> rowLenHistogram(const SparseMatrix* A);

// permuteLongestRowFirst's permutation vector: rows ordered by (length, row
// index) descending -- Python's sort(reverse=True) of (len, i) pairs, so equal
// lengths put the higher row index first.  perm[i] = the row placed at i.
std::vector<uint32_t> longestRowFirstPermutation(const SparseMatrix* A);

// Row i of the result is row perm[i] of A (the permutation-matrix product
// makePermutationMatrixFromVector(perm) * A), as a CSC matrix that owns its
// arrays, row ids ascending within each column (what .tocsc() gives).
SparseMatrix* permuteRows(const SparseMatrix* A, const std::vector<uint32_t>& perm);

inline SparseMatrix* permuteLongestRowFirst(const SparseMatrix* A) {
  return permuteRows(A, longestRowFirstPermutation(A));
}

#endif
