// SpMV: abstract y = A*x operator, the plugin base class of
// software/SpMV.h:8-35.  Non-owning A, x and y; exec() runs one product;
// statKeys()/statInt() expose named counters for the benchmark CSV.
#ifndef SPMV_AMD_SPMV_H_
#define SPMV_AMD_SPMV_H_

#include <string>
#include <vector>

#include "SparseMatrix.h"

class SpMV {
 public:
  SpMV(SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~SpMV();

  virtual bool exec() = 0;

  SparseMatrix* getA() const { return m_A; }
  SpMVData* getX() const { return m_x; }
  SpMVData* getY() const { return m_y; }

  virtual unsigned int statInt(std::string name) = 0;
  virtual std::vector<std::string> statKeys() = 0;

 protected:
  SparseMatrix* m_A;
  SpMVData* m_x;
  SpMVData* m_y;
};

#endif
