// HardwareSpMV: base class of accelerator backends (software/HardwareSpMV.h:8-36).
//
// On the Zynq the two addresses were AXI-Lite MMIO bases (accelerator register
// file and reset register).  MI355X has no MMIO register file, so `aBase`
// points at an in-memory register block whose first 32-bit word is the
// backend signature (what HWSpMVFactory reads, HWSpMVFactory.cpp:22) and
// `aReset` at a 32-bit reset word; both are uintptr_t to hold host pointers.
#ifndef SPMV_AMD_HARDWARESPMV_H_
#define SPMV_AMD_HARDWARESPMV_H_

#include <cstdint>
#include <string>
#include <vector>

#include "SpMV.h"

class HardwareSpMV : public SpMV {
 public:
  HardwareSpMV(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~HardwareSpMV();

  void resetAccelerator();
  // memcmp of y against a golden vector; statInt("diffFromGolden") == 0 iff
  // bit-identical (HardwareSpMV.cpp:37-39).
  void compareGolden(SpMVData* golden);

  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();

  virtual void setThresholds(unsigned int colPtr, unsigned int rowInd, unsigned int nzData, unsigned int inpVec);

 protected:
  volatile uint32_t* m_accelBase;
  volatile uint32_t* m_resetBase;
  int m_diffFromGolden;
  unsigned int m_thres_colPtr;
  unsigned int m_thres_rowInd;
  unsigned int m_thres_nzData;
  unsigned int m_thres_inpVec;

  virtual void init();
  virtual void write();
  virtual void regular();
  virtual void setThresholdRegisters() = 0;
  virtual void setupRegs();
};

#endif
