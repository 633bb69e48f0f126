// HWSpMVFactory: instantiate the backend whose signature sits at aBase
// (software/HWSpMVFactory.h:8-17).  The only backend on MI355X is HIPSpMV.
#ifndef SPMV_AMD_HWSPMVFACTORY_H_
#define SPMV_AMD_HWSPMVFACTORY_H_

#include <cstdint>
#include <string>

#include "HardwareSpMV.h"

class HWSpMVFactory {
 public:
  HWSpMVFactory();
  virtual ~HWSpMVFactory();

  // The backend whose signature is the first 32-bit word at aBase, as a new
  // object the caller deletes; nullptr (and a message on stdout) for an
  // unrecognised signature, where the reference asserts.
  static HardwareSpMV* make(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
  // The backend's short name for the CSV's accType column ("HIPSpMV").
  static std::string name(uintptr_t aBase);
};

#endif
