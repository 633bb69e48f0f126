// csr2csc: stable counting-sort transpose (software/csr2csc.c:11-39).
// The reference signature (int indices, double values; a == nullptr moves the
// pattern only) plus an unsigned/8-byte-word overload used for both f64 and
// u64 matrices.  Symmetric: swapping the roles of rows and columns turns CSC
// into CSR.
#ifndef SPMV_AMD_CSR2CSC_H_
#define SPMV_AMD_CSR2CSC_H_

#include <cstdint>

void csr2csc(int n, int m, int nz, double* a, int* col_idx, int* row_start, double* csc_a, int* row_idx,
             int* col_start);
void csr2csc(uint32_t n, uint32_t m, uint32_t nz, const uint64_t* a, const uint32_t* col_idx,
             const uint32_t* row_start, uint64_t* csc_a, uint32_t* row_idx, uint32_t* col_start);

#endif
