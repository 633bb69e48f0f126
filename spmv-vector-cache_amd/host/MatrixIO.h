// Matrix I/O for the reference's on-disk CSC format and Matrix Market.
//
// The .bin layout is the one matrices/matrixutils.py:187-260 writes and
// software/main.cpp:26-37 reads: <dir>/<name>/<name>-meta.bin (7 x u32
// CompressedSparseMetadata), -indptr.bin (u32[cols+1]), -inds.bin (u32[nz]),
// -data.bin (8-byte values[nz]) and optionally golden.bin (f64[rows] = A*1).
// writeSparseMatrix reproduces the reference files byte for byte, including
// the Zynq DDR base addresses in the metadata (dramBase 0x8000100, 64-byte
// aligned increments, matrixutils.py:9,174-180).
#ifndef SPMV_AMD_MATRIXIO_H_
#define SPMV_AMD_MATRIXIO_H_

#include <string>

#include "SparseMatrix.h"

// Loads <dir>/<name>/<name>-*.bin into arrays the returned matrix owns.  The
// element type is u64 when the name contains "uint64" (the reference's naming
// for its integer fixtures), f64 otherwise.  nullptr on error.
SparseMatrix* loadSparseMatrix(const std::string& dir, const std::string& name);
bool loadGolden(const std::string& path, unsigned int rows, SpMVData* out);
// Matrix Market coordinate file (real/integer/pattern; general/symmetric/
// skew-symmetric) -> CSC with duplicates summed and row ids ascending, as
// scipy's mmread().tocsc() gives (matrixutils.py:163-169).
SparseMatrix* loadMatrixMarket(const std::string& path);
bool writeSparseMatrix(const SparseMatrix* A, const std::string& dir, const std::string& name);
// golden.bin: y = A * ones (matrixutils.py:105-113), f64.
bool writeGolden(const SparseMatrix* A, const std::string& path);

#endif
