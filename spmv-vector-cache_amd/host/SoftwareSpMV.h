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
  // (SoftwareSpMV.cpp:23-39).  Vectors passed in are not owned.
  SoftwareSpMV(SparseMatrix* A, SpMVData* x = 0, SpMVData* y = 0);
  virtual ~SoftwareSpMV();

  // Times maxColSpan, maxAlive and CMS marking of A (SoftwareSpMV.cpp:72-95);
  // A's row ids are left unmarked afterwards.
  void measurePreprocessingTimes();

  // y += A*x in column order; true (the reference's return value)
  virtual bool exec();

  // "rows", "cols", "nz", "spmvtime", "cmstime", "maxAliveTime",
  // "maxColSpanTime", "maxAlive", "maxColSpan"; times in microseconds
  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();

 protected:
  struct Stats {
    unsigned int spmvUs = 0, cmsUs = 0, maxAliveUs = 0, maxColSpanUs = 0;
    unsigned int maxAlive = 0, maxColSpan = 0;
  };
  bool m_ownX = false, m_ownY = false;  // vectors allocated by the constructor
  Stats m_stats;
};

#endif
