/*
 * oracle.h -- CPU restatement of the reference SpMV hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libhipspmv.so,
 * libspmvhost.so, the HIPSpMV backend) links, loads or calls this code.  It is
 * the parity checker used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.
 *
 * Each function restates one reference function; the file:line it follows is
 * given beside it (paths relative to maltanar/spmv-vector-cache).
 *
 * Pinning: the f64 scatter is checked bit-for-bit against every golden.bin the
 * reference ships (matrices/{i64,i1k,i64k,row64k,circuit204}/golden.bin, made
 * by matrices/matrixutils.py:108-113), and the u64 semiring against the
 * known-answer tests of chisel/tests/TestSpMVFrontend.scala:121-143,148-182
 * (see tests/test_oracle.py).  The reference's SpMV loop is not buildable here:
 * software/timer.c needs the ARM-only Xilinx BSP (XScuTimer, software/bsp_lib).
 * software/SparseMatrix.cpp is: `make ref` compiles it into _ref/, and
 * tests/test_oracle_ref.py checks the CMS / maxAlive / maxColSpan /
 * clearRowMarkings restatements below against it bit for bit.
 */
#ifndef SPMV_ORACLE_H_
#define SPMV_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* software/SoftwareSpMV.cpp:50-70 -- y[rowInd[e]] += nzData[e] * x[col],
 * columns ascending, elements ascending; accumulates into the caller's y. */
void oracle_spmv_csc_f64(uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                         const double *vals, const double *x, double *y);

/* Same loop over the integer semiring of chisel/frontend/SemiringOp.scala:74-92
 * (StagedUIntOp with w = 64: product and sum truncated to 64 bits). */
void oracle_spmv_csc_u64(uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                         const uint64_t *vals, const uint64_t *x, uint64_t *y);

/* software/csr2csc.c:11-39 -- stable counting-sort transpose of an n x m CSR
 * matrix into CSC.  8-byte values are moved as opaque words (vals may be NULL:
 * pattern only).  Symmetric: called with (cols, rows, colptr, rowind) it turns
 * CSC into CSR. */
void oracle_csr2csc(uint32_t n, uint32_t m, uint32_t nz, const uint64_t *a, const uint32_t *col_idx,
                    const uint32_t *row_start, uint64_t *csc_a, uint32_t *row_idx, uint32_t *col_start);

/* software/SparseMatrix.cpp:52-90 -- set bit `shift` on the first (reverse = 0)
 * or last (reverse = 1) occurrence of every row index, in place. */
void oracle_mark_row_starts(uint32_t rows, uint32_t nz, uint32_t *inds, int reverse, int shift);

/* software/SparseMatrix.cpp:92-108 (marks inds in place, like the reference). */
uint32_t oracle_max_alive(uint32_t rows, uint32_t nz, uint32_t *inds);

/* software/SparseMatrix.cpp:110-119 */
uint32_t oracle_max_col_span(uint32_t cols, const uint32_t *colptr, const uint32_t *inds);

/* software/SparseMatrix.cpp:121-125 */
void oracle_clear_row_markings(uint32_t nz, uint32_t *inds, uint32_t mask);

/* Times `reps` calls of oracle_spmv_csc_f64 (y zeroed before each) with
 * CLOCK_MONOTONIC around the loop only, mirroring SoftwareSpMV.cpp:57-67.
 * Returns seconds per call. */
double oracle_time_spmv_csc_f64(uint32_t rows, uint32_t cols, const uint32_t *colptr, const uint32_t *rowind,
                                const double *vals, const double *x, double *y, int reps);

#ifdef __cplusplus
}
#endif
/* Row-parallel CSR SpMV on nthreads pthreads (second CPU baseline, bench.py);
 * same bits as oracle_spmv_csc_f64 for column-sorted CSR.  Mean s/exec. */
double oracle_time_spmv_csr_f64_mt(uint32_t rows, const uint32_t *rowptr, const uint32_t *colind,
                                   const double *vals, const double *x, double *y, int reps, int nthreads);

#endif
