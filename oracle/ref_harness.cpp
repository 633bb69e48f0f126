// ref_harness.cpp -- C entry points into the REFERENCE's own
// software/SparseMatrix.cpp, compiled unmodified from /root/reference by
// oracle/Makefile (target `ref`) into oracle/_ref/libref_sparsematrix.so.
//
// TEST INFRASTRUCTURE ONLY: tests/test_oracle_ref.py uses it to check the
// oracle's restatements (oracle.c: mark_row_starts, max_alive, max_col_span,
// clear_row_markings) against the reference code itself.  Nothing in the
// product links or loads it.
//
// Only SparseMatrix.cpp is buildable here: it needs nothing beyond the C++
// standard library.  SoftwareSpMV.cpp (the SpMV loop) includes timer.h, whose
// implementation needs the ARM-only Xilinx BSP (XScuTimer); it stays unbuilt
// and the SpMV itself is pinned by the reference's golden.bin files.
//
// SparseMatrix::fromMemory takes 32-bit addresses (SparseMatrix.cpp:29-50) and
// cannot describe host arrays on x86-64, so a subclass fills the protected
// fields directly -- the same fields fromMemory writes.
#include <cstdint>

#include "SparseMatrix.h"

namespace {

struct HostMatrix : public SparseMatrix {
  HostMatrix(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds) {
    m_rows = rows;
    m_cols = cols;
    m_nz = nz;
    m_indPtrs = colptr;
    m_inds = inds;
    m_nzData = nullptr;  // none of the functions below reads values
    m_rowStartsMarked = false;
  }
};

}  // namespace

extern "C" {

// SparseMatrix::markRowStarts(reverse, shift), in place on inds
void ref_mark_row_starts(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds, int reverse,
                         int shift) {
  HostMatrix m(rows, cols, nz, colptr, inds);
  m.markRowStarts(reverse != 0, shift);
}

// SparseMatrix::maxAlive() (marks inds in place, as the reference does)
uint32_t ref_max_alive(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds) {
  HostMatrix m(rows, cols, nz, colptr, inds);
  return m.maxAlive();
}

// SparseMatrix::maxColSpan()
uint32_t ref_max_col_span(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds) {
  HostMatrix m(rows, cols, nz, colptr, inds);
  return m.maxColSpan();
}

// SparseMatrix::clearRowMarkings(mask), in place on inds
void ref_clear_row_markings(uint32_t rows, uint32_t cols, uint32_t nz, uint32_t* colptr, uint32_t* inds,
                            uint32_t mask) {
  HostMatrix m(rows, cols, nz, colptr, inds);
  m.clearRowMarkings(mask);
}

}  // extern "C"
