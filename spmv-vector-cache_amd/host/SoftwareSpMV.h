// SoftwareSpMV: the CPU golden model (software/SoftwareSpMV.h, .cpp:1-131).
// Column-order scatter over the CSC arrays, y += A*x, single thread.
// Handles f64 and the u64 integer semiring (matrix data type).  Times are
// reported in microseconds (the reference's 333 MHz SCU timer ticks do not
// exist on this host).
#ifndef SPMV_AMD_SOFTWARESPMV_H_
#define SPMV_AMD_SOFTWARESPMV_H_

#include "SpMV.h"

class SoftwareSpMV : public SpMV {
 public:
  // x == nullptr: an all-ones x is allocated; y == nullptr: an all-zero y
  // (SoftwareSpMV.cpp:23-39).
  SoftwareSpMV(SparseMatrix* A, SpMVData* x = 0, SpMVData* y = 0);
  virtual ~SoftwareSpMV();

  void measurePreprocessingTimes();

  virtual bool exec();

  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();

 protected:
  bool m_allocX = false, m_allocY = false;
  unsigned int m_execTime = 0;
  unsigned int m_cmsTime = 0;
  unsigned int m_maxAliveTime = 0;
  unsigned int m_maxColSpanTime = 0;
  unsigned int m_maxAlive = 0;
  unsigned int m_maxColSpan = 0;
};

#endif
