// extern "C" helpers of libspmvhost.so for the Python harness (bench.py,
// tests/): synthetic generators, the product csr2csc and the .bin loader.
// Plain C types only, like include/hipspmv.h.
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "MatrixIO.h"
#include "MatrixOps.h"
#include "Synthetic.h"
#include "csr2csc.h"

extern "C" {

void spmvhost_gen_stripe_csr(uint64_t row0, uint32_t nrows, uint32_t cols, uint32_t k, uint64_t seed_col,
                             uint64_t seed_val, uint32_t* rowptr, uint32_t* colind, double* vals) {
  genStripeCSR(row0, nrows, cols, k, seed_col, seed_val, rowptr, colind, vals);
}

void spmvhost_gen_vector(uint64_t n, uint64_t seed, double* out) {
  const unsigned nt = n > (1u << 20) ? hostThreads() : 1;
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < nt; ++t)
    pool.emplace_back([=] {
      for (uint64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) out[i] = uniform11(splitmix64_at(seed, i));
    });
  for (auto& th : pool) th.join();
}

uint64_t spmvhost_splitmix64_at(uint64_t seed, uint64_t i) { return splitmix64_at(seed, i); }

// Fills caller arrays sized for the upper bound (rowptr: 2^scale+1, colind/vals:
// edge_factor*2^scale); returns the nnz after summing duplicates.
uint64_t spmvhost_gen_rmat_csr(uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t* rowptr,
                               uint32_t* colind, double* vals) {
  std::vector<uint32_t> rp, ci;
  std::vector<double> v;
  const uint64_t nnz = genRmatCSR(scale, edge_factor, seed, 0.57, 0.19, 0.19, rp, ci, v);
  std::memcpy(rowptr, rp.data(), sizeof(uint32_t) * rp.size());
  std::memcpy(colind, ci.data(), sizeof(uint32_t) * nnz);
  std::memcpy(vals, v.data(), sizeof(double) * nnz);
  return nnz;
}

// Rows [row0, row1) of the R-MAT matrix.  Copies into the caller's arrays
// (rowptr: row1-row0+1, colind/vals: cap) when nnz <= cap; always returns nnz.
uint64_t spmvhost_gen_rmat_rows(uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t row0, uint32_t row1,
                                uint32_t* rowptr, uint32_t* colind, double* vals, uint64_t cap) {
  std::vector<uint32_t> rp, ci;
  std::vector<double> v;
  const uint64_t nnz = genRmatCSRRows(scale, edge_factor, seed, 0.57, 0.19, 0.19, row0, row1, rp, ci, v);
  if (nnz <= cap) {
    std::memcpy(rowptr, rp.data(), sizeof(uint32_t) * rp.size());
    std::memcpy(colind, ci.data(), sizeof(uint32_t) * nnz);
    std::memcpy(vals, v.data(), sizeof(double) * nnz);
  }
  return nnz;
}

void spmvhost_gen_rmat_row_counts(uint32_t scale, uint32_t edge_factor, uint64_t seed, uint32_t* counts) {
  genRmatRowCounts(scale, edge_factor, seed, 0.57, 0.19, 0.19, counts);
}

void spmvhost_partition_row_counts(const uint32_t* counts, uint32_t rows, uint32_t parts, uint32_t* bounds) {
  partitionRowCounts(counts, rows, parts, bounds);
}

void spmvhost_csr2csc(uint32_t n, uint32_t m, uint32_t nz, const uint64_t* a, const uint32_t* col_idx,
                      const uint32_t* row_start, uint64_t* csc_a, uint32_t* row_idx, uint32_t* col_start) {
  csr2csc(n, m, nz, a, col_idx, row_start, csc_a, row_idx, col_start);
}

void spmvhost_partition_rows(const uint32_t* rowptr, uint32_t rows, uint32_t parts, uint32_t* bounds) {
  partitionRows(rowptr, rows, parts, bounds);
}

// Loads <dir>/<name>; copies into caller arrays when they are non-null, and
// always reports the dimensions.  Returns 0 on success.
int spmvhost_load_matrix(const char* dir, const char* name, uint32_t* dims /*rows, cols, nz, is_u64*/,
                         uint32_t* colptr, uint32_t* rowind, uint64_t* vals) try {
  SparseMatrix* A = loadSparseMatrix(dir, name);
  if (!A) return 1;
  dims[0] = A->getRows();
  dims[1] = A->getCols();
  dims[2] = A->getNz();
  dims[3] = A->getDataType() == SPMV_U64;
  if (colptr) std::memcpy(colptr, A->getIndPtrs(), 4ull * (A->getCols() + 1));
  if (rowind) std::memcpy(rowind, A->getInds(), 4ull * A->getNz());
  if (vals) std::memcpy(vals, A->getNzData(), 8ull * A->getNz());
  delete A;
  return 0;
} catch (...) {  // nothing throws across the C boundary
  return 3;
}

// Row-length histogram (matrixutils.py:116-126, MatrixOps.h): writes up to
// cap (length, count) pairs in ascending length; returns the number of pairs.
uint32_t spmvhost_row_len_histogram(uint32_t rows, uint32_t cols, uint32_t nz, const uint32_t* colptr,
                                    const uint32_t* rowind, uint32_t* lens, uint32_t* counts, uint32_t cap) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, const_cast<uint32_t*>(colptr),
                                             const_cast<uint32_t*>(rowind), nullptr);
  const auto h = rowLenHistogram(A);
  delete A;
  uint32_t i = 0;
  for (const auto& kv : h) {
    if (i < cap) {
      lens[i] = kv.first;
      counts[i] = kv.second;
    }
    ++i;
  }
  return i;
}

// permuteLongestRowFirst (matrixutils.py:140-158) on CSC arrays: perm[rows]
// and the permuted CSC (colptr[cols+1], rowind[nz], vals[nz] 8-byte words).
void spmvhost_permute_longest_row_first(uint32_t rows, uint32_t cols, uint32_t nz, const uint32_t* colptr,
                                        const uint32_t* rowind, const uint64_t* vals, uint32_t* perm,
                                        uint32_t* colptr_out, uint32_t* rowind_out, uint64_t* vals_out) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, const_cast<uint32_t*>(colptr),
                                             const_cast<uint32_t*>(rowind),
                                             reinterpret_cast<SpMVData*>(const_cast<uint64_t*>(vals)));
  const std::vector<uint32_t> p = longestRowFirstPermutation(A);
  SparseMatrix* B = permuteRows(A, p);
  std::memcpy(perm, p.data(), 4ull * rows);
  std::memcpy(colptr_out, B->getIndPtrs(), 4ull * (cols + 1));
  std::memcpy(rowind_out, B->getInds(), 4ull * nz);
  std::memcpy(vals_out, B->getNzData(), 8ull * nz);
  delete B;
  delete A;
}

// SparseMatrix's preprocessing helpers (host/SparseMatrix.cpp, the statistics
// SoftwareSpMV::measurePreprocessingTimes reports) on caller CSC arrays, in
// place on inds like the reference; tests/test_oracle_ref.py checks them
// against the reference's own SparseMatrix.cpp.
void spmvhost_mark_row_starts(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds,
                              int reverse, int shift) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, colptr, inds, nullptr);
  A->markRowStarts(reverse != 0, shift);
  delete A;
}

uint32_t spmvhost_max_alive(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, colptr, inds, nullptr);
  const uint32_t v = A->maxAlive();
  delete A;
  return v;
}

uint32_t spmvhost_max_col_span(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, colptr, inds, nullptr);
  const uint32_t v = A->maxColSpan();
  delete A;
  return v;
}

void spmvhost_clear_row_markings(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds,
                                 uint32_t mask) {
  SparseMatrix* A = SparseMatrix::fromArrays(rows, cols, nz, colptr, inds, nullptr);
  A->clearRowMarkings(mask);
  delete A;
}

// Matrix Market -> reference .bin files (+ golden.bin) under <outdir>/<name>/,
// the job of matrices/matrixutils.py:187-260 and :108-113; with permute, rows
// are reordered longest first before writing (:149-158).  Returns 0 on success.
int spmvhost_convert_mtx(const char* mtx_path, const char* outdir, const char* name, int write_golden,
                         int permute) try {
  SparseMatrix* A = loadMatrixMarket(mtx_path);
  if (!A) return 1;
  if (permute) {
    SparseMatrix* B = permuteLongestRowFirst(A);
    delete A;
    A = B;
  }
  bool ok = writeSparseMatrix(A, outdir, name);
  if (ok && write_golden) ok = writeGolden(A, std::string(outdir) + "/" + name + "/golden.bin");
  delete A;
  return ok ? 0 : 2;
} catch (...) {
  return 3;
}

}  // extern "C"
