#include "SparseMatrix.h"

#include <iostream>
#include <vector>

SparseMatrix::SparseMatrix() {}

SparseMatrix::~SparseMatrix() {
  if (m_owned) {
    delete[] m_indPtrs;
    delete[] m_inds;
    delete[] m_nzData;
  }
}

void SparseMatrix::printSummary() {
  std::cout << "Matrix summary\nname = " << m_name << "\n#rows = " << m_rows << "\n#cols = " << m_cols
            << "\n#nz = " << m_nz << std::endl;
}

bool SparseMatrix::isSquare() { return m_rows == m_cols; }

SparseMatrix* SparseMatrix::fromMemory(const CompressedSparseMetadata* meta, uintptr_t addrBias) {
  if (!meta || meta->numRows == 0 || meta->numCols == 0 || meta->numNZ == 0) {
    std::cerr << "Error: matrix metadata at " << std::hex << (uintptr_t)meta << std::dec << " is invalid"
              << std::endl;
    return nullptr;
  }
  SparseMatrix* m = new SparseMatrix();
  m->m_rows = meta->numRows;
  m->m_cols = meta->numCols;
  m->m_nz = meta->numNZ;
  m->m_indPtrs = reinterpret_cast<SpMVIndex*>(addrBias + meta->indPtrBase);
  m->m_inds = reinterpret_cast<SpMVIndex*>(addrBias + meta->indBase);
  m->m_nzData = reinterpret_cast<SpMVData*>(addrBias + meta->nzDataBase);
  return m;
}

SparseMatrix* SparseMatrix::fromArrays(unsigned int rows, unsigned int cols, unsigned int nz, SpMVIndex* indPtrs,
                                       SpMVIndex* inds, SpMVData* nzData, SpMVDataType type, bool takeOwnership) {
  SparseMatrix* m = new SparseMatrix();
  m->m_rows = rows;
  m->m_cols = cols;
  m->m_nz = nz;
  m->m_indPtrs = indPtrs;
  m->m_inds = inds;
  m->m_nzData = nzData;
  m->m_type = type;
  m->m_owned = takeOwnership;
  return m;
}

// Walk the row indices forwards (first touch) or backwards (last touch) and
// set bit `shift` on the first occurrence of each row; a bitmap of seen rows
// is indexed with the low 30 bits so earlier markings do not alias
// (SparseMatrix.cpp:52-90).
void SparseMatrix::markRowStarts(const bool reverse, const int shift) {
  std::vector<uint32_t> seen(m_rows / 32 + 1, 0u);
  for (SpMVIndex n = 0; n < m_nz; ++n) {
    const SpMVIndex e = reverse ? m_nz - 1 - n : n;
    const SpMVIndex row = m_inds[e] & 0x3FFFFFFFu;
    uint32_t& word = seen[row >> 5];
    const uint32_t bit = 1u << (row & 31);
    if (!(word & bit)) {
      word |= bit;
      m_inds[e] |= 1u << shift;
    }
  }
  m_rowStartsMarked = true;
  ++m_version;
}

// Largest number of rows that have been touched but not finished at any
// point of the column-order stream (SparseMatrix.cpp:92-108).
unsigned int SparseMatrix::maxAlive() {
  markRowStarts(false, 31);
  markRowStarts(true, 30);
  unsigned int best = 0, alive = 0;
  for (SpMVIndex e = 0; e < m_nz; ++e) {
    if (m_inds[e] & (1u << 31)) ++alive;
    if (m_inds[e] & (1u << 30)) --alive;
    if (alive > best) best = alive;
  }
  return best;
}

// Largest row-id distance between the first and last entry of a column
// (SparseMatrix.cpp:110-119).  A leading empty column contributes 0 instead
// of reading before the index array.
unsigned int SparseMatrix::maxColSpan() {
  unsigned int best = 0;
  // SparseMatrix.cpp:110-119, also for empty columns (they read the
  // neighbouring columns' entries); reads that would leave [0, nz) -- the
  // reference's undefined cases -- contribute nothing.
  for (SpMVIndex c = 0; c < m_cols; ++c) {
    if (m_indPtrs[c + 1] == 0 || m_indPtrs[c] >= m_nz || m_indPtrs[c + 1] > m_nz) continue;
    const unsigned int span = m_inds[m_indPtrs[c + 1] - 1] - m_inds[m_indPtrs[c]];
    if (span > best) best = span;
  }
  return best;
}

void SparseMatrix::clearRowMarkings(const unsigned int mask) {
  for (SpMVIndex e = 0; e < m_nz; ++e) m_inds[e] &= mask;
  m_rowStartsMarked = false;
  ++m_version;
}
