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
  // The operator keeps the three pointers; it never frees them (SpMV.cpp:10-12).
  SpMV(SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~SpMV();

  // One y = A*x pass with the backend's semantics; true on success.
  virtual bool exec() = 0;

  // Operands as given at construction (or allocated by the subclass).
  SparseMatrix* getA() const { return m_A; }
  SpMVData* getX() const { return m_x; }
  SpMVData* getY() const { return m_y; }

  // Named 32-bit counters; statKeys() lists the names in CSV column order
  // (main.cpp:49-66 prints them), statInt() returns 0 for an unknown name.
  virtual unsigned int statInt(std::string name) = 0;
  virtual std::vector<std::string> statKeys() = 0;

 protected:
  SparseMatrix* m_A;  // not owned
  SpMVData* m_x;      // input vector, cols entries
  SpMVData* m_y;      // output vector, rows entries
};

#endif
