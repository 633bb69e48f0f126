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
  // aBase: the backend's register block (word 0 = signature); aReset: its
  // reset word.  Neither is owned.
  HardwareSpMV(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~HardwareSpMV();

  // Pulse the reset word; marks the result as not yet compared.
  void resetAccelerator();
  // memcmp of y against a golden vector; statInt("diffFromGolden") == 0 iff
  // bit-identical (HardwareSpMV.cpp:37-39).
  void compareGolden(SpMVData* golden);

  // "diffFromGolden", "rows", "cols", "nz" (HardwareSpMV.cpp:41-61)
  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();

  // Stream-FIFO throttle thresholds of the FPGA backends (default 128 each);
  // a backend without FIFOs keeps them as statistics only.
  virtual void setThresholds(unsigned int colPtr, unsigned int rowInd, unsigned int nzData, unsigned int inpVec);

 protected:
  struct Thresholds {
    uint32_t colPtr = 128, rowInd = 128, nzData = 128, inpVec = 128;
  };
  volatile uint32_t* m_accelBase;  // register block (signature at word 0)
  volatile uint32_t* m_resetBase;  // reset word
  int m_diffFromGolden = 1;        // memcmp result; 1 until compareGolden runs
  Thresholds m_thres;

  // exec() phases of a backend, in the order HardwareSpMVNewCache.cpp:78-88
  // calls them: setupRegs (program the matrix), init, regular (the SpMV),
  // write (y back to the caller).
  virtual void setupRegs();
  virtual void init();
  virtual void regular();
  virtual void write();
  virtual void setThresholdRegisters() = 0;
};

#endif
