// SparseMatrix: the CSC container the SpMV plugins operate on.
//
// Restates software/SparseMatrix.h:1-70 / SparseMatrix.cpp:1-125 of
// maltanar/spmv-vector-cache for a 64-bit host.  Same element types, same
// getters, same cold-miss-skip (CMS) marking helpers.  Differences:
//  * fromMemory() takes the metadata block plus the address bias that maps its
//    32-bit Zynq DDR addresses (SparseMatrix.cpp:29-50) onto host memory;
//  * fromArrays() wraps caller arrays (optionally taking ownership);
//  * the element type is recorded (f64, or the u64 integer semiring of
//    chisel/frontend/SemiringOp.scala:74-92 stored in the same 8-byte words).
#ifndef SPMV_AMD_SPARSEMATRIX_H_
#define SPMV_AMD_SPARSEMATRIX_H_

#include <cstdint>
#include <string>

typedef unsigned int SpMVIndex;  // SparseMatrix.h:5
typedef double SpMVData;         // SparseMatrix.h:6

// 28-byte metadata block of a matrix on disk / in memory (SparseMatrix.h:8-16,
// written by matrices/matrixutils.py:200-250).
typedef struct {
  unsigned int numRows;
  unsigned int numCols;
  unsigned int numNZ;
  unsigned int startingRow;
  unsigned int indPtrBase;
  unsigned int indBase;
  unsigned int nzDataBase;
} CompressedSparseMetadata;

enum SpMVDataType { SPMV_F64 = 0, SPMV_U64 = 1 };

class SparseMatrix {
 public:
  SparseMatrix();
  virtual ~SparseMatrix();

  void printSummary();
  bool isSquare();

  void setName(std::string name) { m_name = name; }
  std::string getName() { return m_name; }

  // metadata at `meta`; each base address field + addrBias is a host pointer.
  // Returns nullptr (and reports on stderr) for an empty/invalid block, like
  // the reference.
  static SparseMatrix* fromMemory(const CompressedSparseMetadata* meta, uintptr_t addrBias);
  // CSC arrays (indPtrs[cols+1], inds[nz], nzData[nz]); with takeOwnership the
  // matrix delete[]s them.
  static SparseMatrix* fromArrays(unsigned int rows, unsigned int cols, unsigned int nz, SpMVIndex* indPtrs,
                                  SpMVIndex* inds, SpMVData* nzData, SpMVDataType type = SPMV_F64,
                                  bool takeOwnership = false);

  // CMS helpers (SparseMatrix.cpp:52-125): mark first (or, reversed, last)
  // touch of each row with bit `shift` of its row index, in place.
  void markRowStarts(const bool reverse = false, const int shift = 31);
  unsigned int maxAlive();
  unsigned int maxColSpan();
  void clearRowMarkings(const unsigned int mask);

  unsigned int getRows() const { return m_rows; }
  unsigned int getCols() const { return m_cols; }
  unsigned int getNz() const { return m_nz; }
  SpMVIndex* getIndPtrs() const { return m_indPtrs; }
  SpMVIndex* getInds() const { return m_inds; }
  SpMVData* getNzData() const { return m_nzData; }
  SpMVDataType getDataType() const { return m_type; }
  void setDataType(SpMVDataType t) { m_type = t; }
  bool rowStartsMarked() const { return m_rowStartsMarked; }
  // bumped by every in-place mutation; backends caching a device copy of the
  // matrix compare it to decide whether to rebuild
  uint64_t version() const { return m_version; }

 protected:
  unsigned int m_rows = 0;
  unsigned int m_cols = 0;
  unsigned int m_nz = 0;
  SpMVIndex* m_indPtrs = nullptr;
  SpMVIndex* m_inds = nullptr;
  SpMVData* m_nzData = nullptr;
  std::string m_name;
  bool m_rowStartsMarked = false;
  SpMVDataType m_type = SPMV_F64;
  bool m_owned = false;
  uint64_t m_version = 0;
};

#endif
