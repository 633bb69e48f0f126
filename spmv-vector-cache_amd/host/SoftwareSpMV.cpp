#include "SoftwareSpMV.h"

#include <chrono>
#include <cstdint>
#include <cstring>
#include <iostream>

namespace {
using Clock = std::chrono::steady_clock;
unsigned int micros_since(Clock::time_point t0) {
  return (unsigned int)std::chrono::duration_cast<std::chrono::microseconds>(Clock::now() - t0).count();
}

// y[rowInd[e]] += nzData[e] * x[col], columns ascending, elements ascending:
// the loop of SoftwareSpMV.cpp:59-64, for either semiring.
template <typename T>
void csc_scatter(unsigned int cols, const SpMVIndex* colPtr, const SpMVIndex* rowInd, const T* nz, const T* x,
                 T* y) {
  for (unsigned int c = 0; c < cols; ++c) {
    const T xc = x[c];
    const SpMVIndex stop = colPtr[c + 1];
    for (SpMVIndex e = colPtr[c]; e < stop; ++e) {
      const T prod = nz[e] * xc;  // rounded before the add (built with -ffp-contract=off)
      y[rowInd[e]] += prod;
    }
  }
}
}  // namespace

SoftwareSpMV::SoftwareSpMV(SparseMatrix* A, SpMVData* x, SpMVData* y) : SpMV(A, x, y) {
  if (!A) {
    std::cerr << "Invalid matrix for SoftwareSpMV!" << std::endl;
    return;
  }
  const bool u64 = A->getDataType() == SPMV_U64;
  if (!x) {
    m_ownX = true;
    m_x = new SpMVData[A->getCols()];
    for (unsigned int i = 0; i < A->getCols(); ++i) {
      if (u64) {
        const uint64_t one = 1;
        std::memcpy(&m_x[i], &one, sizeof one);
      } else {
        m_x[i] = 1.0;
      }
    }
  }
  if (!y) {
    m_ownY = true;
    m_y = new SpMVData[A->getRows()];
    std::memset(m_y, 0, sizeof(SpMVData) * A->getRows());  // +0.0 and integer 0 share the bit pattern
  }
}

SoftwareSpMV::~SoftwareSpMV() {
  if (m_ownX) delete[] m_x;
  if (m_ownY) delete[] m_y;
}

bool SoftwareSpMV::exec() {
  const auto t0 = Clock::now();
  if (m_A->getDataType() == SPMV_U64)
    csc_scatter<uint64_t>(m_A->getCols(), m_A->getIndPtrs(), m_A->getInds(),
                          reinterpret_cast<const uint64_t*>(m_A->getNzData()),
                          reinterpret_cast<const uint64_t*>(m_x), reinterpret_cast<uint64_t*>(m_y));
  else
    csc_scatter<double>(m_A->getCols(), m_A->getIndPtrs(), m_A->getInds(), m_A->getNzData(), m_x, m_y);
  m_stats.spmvUs = micros_since(t0);
  return true;
}

// SoftwareSpMV.cpp:72-94: time maxColSpan, maxAlive and CMS marking, then
// strip the marks again so a later exec() sees clean row ids.
void SoftwareSpMV::measurePreprocessingTimes() {
  const unsigned int keep = ~((1u << 31) | (1u << 30));
  auto t0 = Clock::now();
  m_stats.maxColSpan = m_A->maxColSpan();
  m_stats.maxColSpanUs = micros_since(t0);
  t0 = Clock::now();
  m_stats.maxAlive = m_A->maxAlive();
  m_stats.maxAliveUs = micros_since(t0);
  m_A->clearRowMarkings(keep);
  t0 = Clock::now();
  m_A->markRowStarts();
  m_stats.cmsUs = micros_since(t0);
  m_A->clearRowMarkings(keep);
}

std::vector<std::string> SoftwareSpMV::statKeys() {
  return {"rows", "cols", "nz", "spmvtime", "cmstime", "maxAliveTime", "maxColSpanTime", "maxAlive", "maxColSpan"};
}

unsigned int SoftwareSpMV::statInt(std::string name) {
  if (name == "rows") return m_A->getRows();
  if (name == "cols") return m_A->getCols();
  if (name == "nz") return m_A->getNz();
  if (name == "spmvtime") return m_stats.spmvUs;
  if (name == "cmstime") return m_stats.cmsUs;
  if (name == "maxAliveTime") return m_stats.maxAliveUs;
  if (name == "maxColSpanTime") return m_stats.maxColSpanUs;
  if (name == "maxAlive") return m_stats.maxAlive;
  if (name == "maxColSpan") return m_stats.maxColSpan;
  return 0;
}
