/*
 * oracle.c -- CPU restatement of the reference SpMV hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the parity checker for tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product never
 * links or calls it.  Built with -ffp-contract=off so that, like the
 * reference's x86 build of SoftwareSpMV.cpp, every product is rounded before it
 * is added (no FMA).
 */
#include "oracle.h"

#include <stdlib.h>
#include <pthread.h>
#include <string.h>
#include <time.h>

/* software/SoftwareSpMV.cpp:50-70; hot loop :59-64. */
void oracle_spmv_csc_f64(uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                         const double *vals, const double *x, double *y) {
  for (uint32_t col = 0; col < cols; col++) {
    const double inp = x[col];
    for (uint32_t e = colptr[col]; e < colptr[col + 1]; e++) y[rowind[e]] += vals[e] * inp;
  }
}

/* Same traversal; integer semiring of chisel/frontend/SemiringOp.scala:74-92
 * (OpMulCombinatorial / OpAddCombinatorial at :35-46 feeding SystolicReg(64),
 * which keeps the low 64 bits).  C unsigned arithmetic wraps mod 2^64. */
void oracle_spmv_csc_u64(uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                         const uint64_t *vals, const uint64_t *x, uint64_t *y) {
  for (uint32_t col = 0; col < cols; col++) {
    const uint64_t inp = x[col];
    for (uint32_t e = colptr[col]; e < colptr[col + 1]; e++) y[rowind[e]] += vals[e] * inp;
  }
}

/* software/csr2csc.c:11-39: count column lengths, prefix-sum, scatter row by
 * row (stable), then shift the pointers back by one. */
void oracle_csr2csc(uint32_t n, uint32_t m, uint32_t nz, const uint64_t *a, const uint32_t *col_idx,
                    const uint32_t *row_start, uint64_t *csc_a, uint32_t *row_idx, uint32_t *col_start) {
  for (uint32_t i = 0; i <= m; i++) col_start[i] = 0;
  for (uint32_t i = 0; i < nz; i++) col_start[col_idx[i] + 1]++;
  for (uint32_t i = 0; i < m; i++) col_start[i + 1] += col_start[i];
  for (uint32_t i = 0; i < n; i++) {
    for (uint32_t j = row_start[i]; j < row_start[i + 1]; j++) {
      const uint32_t k = col_idx[j];
      const uint32_t l = col_start[k]++;
      row_idx[l] = i;
      if (a) csc_a[l] = a[j];
    }
  }
  for (uint32_t i = m; i > 0; i--) col_start[i] = col_start[i - 1];
  col_start[0] = 0;
}

/* software/SparseMatrix.cpp:52-90.  Row ids are masked with 0x3FFFFFFF before
 * use, exactly as the reference does, so earlier markings do not alias. */
void oracle_mark_row_starts(uint32_t rows, uint32_t nz, uint32_t *inds, int reverse, int shift) {
  const uint32_t words = rows / 32 + 1;
  uint32_t *seen = (uint32_t *)calloc(words, sizeof(uint32_t));
  for (uint32_t n = 0; n < nz; n++) {
    const uint32_t e = reverse ? nz - 1 - n : n;
    const uint32_t row = inds[e] & 0x3FFFFFFFu;
    const uint32_t w = row / 32, bit = 1u << (row % 32);
    if ((seen[w] & bit) == 0) {
      seen[w] |= bit;
      inds[e] |= 1u << shift;
    }
  }
  free(seen);
}

/* software/SparseMatrix.cpp:92-108: bit 31 = first touch of a row, bit 30 =
 * last touch; the running count of rows "alive" between the two, maximised. */
uint32_t oracle_max_alive(uint32_t rows, uint32_t nz, uint32_t *inds) {
  oracle_mark_row_starts(rows, nz, inds, 0, 31);
  oracle_mark_row_starts(rows, nz, inds, 1, 30);
  uint32_t best = 0, alive = 0;
  for (uint32_t e = 0; e < nz; e++) {
    if (inds[e] & (1u << 31)) alive += 1;
    if (inds[e] & (1u << 30)) alive -= 1;
    if (alive > best) best = alive;
  }
  return best;
}

/* software/SparseMatrix.cpp:110-119.  The reference reads
 * inds[colptr[c+1]-1] - inds[colptr[c]] with unsigned wrap-around, also for
 * empty columns (where it reads the neighbouring columns' entries); restated
 * as is, except that an empty column whose reads would leave [0, nnz) -- a
 * leading one reads inds[-1], a trailing one inds[nnz] -- contributes 0
 * (undefined in the reference). */
uint32_t oracle_max_col_span(uint32_t cols, const uint32_t *colptr, const uint32_t *inds) {
  uint32_t best = 0;
  const uint32_t nz = colptr[cols];
  for (uint32_t c = 0; c < cols; c++) {
    if (colptr[c + 1] == 0 || colptr[c] >= nz || colptr[c + 1] > nz) continue;
    const uint32_t span = inds[colptr[c + 1] - 1] - inds[colptr[c]];
    if (span > best) best = span;
  }
  return best;
}

/* software/SparseMatrix.cpp:121-125 */
void oracle_clear_row_markings(uint32_t nz, uint32_t *inds, uint32_t mask) {
  for (uint32_t e = 0; e < nz; e++) inds[e] &= mask;
}

double oracle_time_spmv_csc_f64(uint32_t rows, uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                                const double *vals, const double *x, double *y, int reps) {
  double total = 0.0;
  for (int r = 0; r < reps; r++) {
    memset(y, 0, sizeof(double) * rows);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_spmv_csc_f64(cols, colptr, rowind, vals, x, y);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    total += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  }
  return reps > 0 ? total / reps : 0.0;
}

/* Second CPU baseline ("optionally, an OpenMP CSR
 * row-parallel CPU run on all cores"): rows split into nthreads contiguous
 * nnz-balanced ranges, one pthread each, every row summed sequentially in its
 * CSR order -- for column-sorted CSR the same order, hence the same bits, as
 * SoftwareSpMV's column scatter.  Returns the mean seconds per exec. */
typedef struct {
  const uint32_t *rowptr, *colind;
  const double *vals, *x;
  double *y;
  uint32_t r0, r1;
} csr_job_t;

static void *csr_rows(void *arg) {
  const csr_job_t *j = (const csr_job_t *)arg;
  for (uint32_t r = j->r0; r < j->r1; r++) {
    double acc = 0.0;
    for (uint32_t e = j->rowptr[r]; e < j->rowptr[r + 1]; e++) {
      const double p = j->vals[e] * j->x[j->colind[e]];
      acc = acc + p;
    }
    j->y[r] = acc;
  }
  return NULL;
}

double oracle_time_spmv_csr_f64_mt(uint32_t rows, const uint32_t *rowptr, const uint32_t *colind,
                                   const double *vals, const double *x, double *y, int reps, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  csr_job_t jobs[256];
  pthread_t th[256];
  const uint64_t nnz = rowptr[rows];
  uint32_t r = 0;
  for (int t = 0; t < nthreads; t++) {
    const uint64_t target = nnz * (uint64_t)(t + 1) / (uint64_t)nthreads;
    const uint32_t r0 = r;
    while (r < rows && (t == nthreads - 1 || rowptr[r + 1] <= target)) r++;
    jobs[t] = (csr_job_t){rowptr, colind, vals, x, y, r0, t == nthreads - 1 ? rows : r};
  }
  double total = 0.0;
  for (int k = 0; k < reps; k++) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, csr_rows, &jobs[t]);
    csr_rows(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    total += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  }
  return reps > 0 ? total / reps : 0.0;
}
