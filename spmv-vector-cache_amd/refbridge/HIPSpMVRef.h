// HIPSpMVRef -- the HIP backend as a maintainer of the REFERENCE would add it
// (INTEGRATION.md section B): a subclass of the reference's own HardwareSpMV
// (ref:software/HardwareSpMV.h:8-36), compiled against the reference headers
// unchanged, driving libhipspmv.so through its C ABI (include/hipspmv.h).
//
// This repo's own restated plugin surface (spmv-vector-cache_amd/host/) widens
// aBase/aReset to uintptr_t; this file keeps the reference's `unsigned int`
// addresses instead, so the register block must sit below 4 GiB (the bridge
// driver maps it with MAP_32BIT).  Register block layout, 32-bit words at
// aBase (the reference reads its accelerator signature at word 0,
// HWSpMVFactory.cpp:22):
//   0 signature (HIPSpMVRef::expSignature(), "MI35")
//   1 device    2 mode (HIPSPMV_MODE_*)   3 kernel (HIPSPMV_KERNEL_*)
//   4 beta (1 = the reference's y += A*x)  5 dtype (HIPSPMV_F64 / HIPSPMV_U64)
// and the reset word at aReset (HardwareSpMV::resetAccelerator pulses it).
#ifndef HIPSPMVREF_H_
#define HIPSPMVREF_H_

#include <stdint.h>

#include <string>
#include <vector>

#include "HardwareSpMV.h"  // the reference's (ref:software/HardwareSpMV.h)
#include "hipspmv.h"

struct HIPSpMVRefRegs {
  uint32_t signature, device, mode, kernel, beta, dtype;
};

class HIPSpMVRef : public HardwareSpMV {
 public:
  // the value the factory branch compares against (ref:software/HWSpMVFactory.cpp:24-31)
  static unsigned int expSignature() { return 0x4D493335u; }

  HIPSpMVRef(unsigned int aBase, unsigned int aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~HIPSpMVRef();

  // the phases of ref:software/HardwareSpMVNewCache.cpp:78-88; true on success
  // (the reference's hardware backends return false, main.cpp:245 ignores it)
  virtual bool exec();

  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();

 protected:
  virtual void init();
  virtual void write();
  virtual void regular();
  virtual void setupRegs();
  virtual void setThresholdRegisters();

 private:
  volatile HIPSpMVRefRegs* regs() const { return (volatile HIPSpMVRefRegs*)m_accelBase; }
  uint64_t stat64(const char* key);
  hipspmv_t* m_h;
  int m_status;
};

// The branches a maintainer adds to HWSpMVFactory::make / ::name
// (ref:software/HWSpMVFactory.cpp:20-57): the HIP backend for its signature,
// nullptr / "" for any other (the reference factory's own branches follow).
HardwareSpMV* makeHIPSpMVRef(unsigned int aBase, unsigned int aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
std::string nameHIPSpMVRef(unsigned int aBase);

#endif  // HIPSPMVREF_H_
