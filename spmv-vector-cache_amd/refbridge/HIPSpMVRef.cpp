// HIPSpMVRef: see HIPSpMVRef.h.  Built only against the reference tree
// (oracle/Makefile target `refbridge`); the product is libhipspmv.so.
#include "HIPSpMVRef.h"

#include <iostream>

HIPSpMVRef::HIPSpMVRef(unsigned int aBase, unsigned int aReset, SparseMatrix* A, SpMVData* x, SpMVData* y)
    : HardwareSpMV(aBase, aReset, A, x, y), m_h(0), m_status(0) {}

HIPSpMVRef::~HIPSpMVRef() {
  if (m_h) hipspmv_destroy(m_h);
}

// setupRegs: the reference programs base addresses and thresholds
// (HardwareSpMV.cpp setupRegs -> setThresholdRegisters); here the matrix goes
// to the device once per backend instance (main.cpp:236 makes one per matrix).
void HIPSpMVRef::setupRegs() {
  HardwareSpMV::setupRegs();
  if (m_status || m_h) return;
  m_status = hipspmv_create(m_A->getIndPtrs(), m_A->getInds(), m_A->getNzData(), m_A->getRows(), m_A->getCols(),
                            m_A->getNz(), (int)regs()->dtype, (int)regs()->device, &m_h);
  if (m_status) {
    std::cerr << "HIPSpMVRef: create failed: " << hipspmv_strerror(m_status) << " (" << hipspmv_last_error() << ")"
              << std::endl;
    m_h = 0;
    return;
  }
  if (regs()->kernel != HIPSPMV_KERNEL_AUTO) m_status = hipspmv_set_option(m_h, "kernel", (int64_t)regs()->kernel);
}

void HIPSpMVRef::init() { HardwareSpMV::init(); }

// regular: x up, the kernel, y back, synchronously (the reference busy-waits
// on the accelerator's done flag, HardwareSpMVNewCache.cpp:90-101)
void HIPSpMVRef::regular() {
  HardwareSpMV::regular();
  if (m_status || !m_h) return;
  m_status = hipspmv_exec(m_h, m_x, m_y, (int)regs()->beta, (int)regs()->mode);
  if (m_status)
    std::cerr << "HIPSpMVRef: exec failed: " << hipspmv_strerror(m_status) << " (" << hipspmv_last_error() << ")"
              << std::endl;
}

void HIPSpMVRef::write() { HardwareSpMV::write(); }

// no stream FIFOs to throttle: setThresholds() values are kept by the base
// class and reported as statistics only
void HIPSpMVRef::setThresholdRegisters() {}

bool HIPSpMVRef::exec() {
  m_status = 0;
  resetAccelerator();
  setupRegs();
  init();
  regular();
  write();
  return m_status == 0;
}

uint64_t HIPSpMVRef::stat64(const char* key) {
  uint64_t v = 0;
  if (m_h && hipspmv_stat(m_h, key, &v) == HIPSPMV_OK) return v;
  return 0;
}

std::vector<std::string> HIPSpMVRef::statKeys() {
  std::vector<std::string> keys = HardwareSpMV::statKeys();
  const char* more[] = {"kernelTimeUs", "setupTimeUs", "h2dTimeUs", "d2hTimeUs", "algKBytes", "mode", "kernel",
                        "device", "error"};
  for (const char* k : more) keys.push_back(k);
  return keys;
}

unsigned int HIPSpMVRef::statInt(std::string name) {
  if (name == "kernelTimeUs") return (unsigned int)(stat64("kernel_ns") / 1000);
  if (name == "setupTimeUs") return (unsigned int)(stat64("setup_ns") / 1000);
  if (name == "h2dTimeUs") return (unsigned int)(stat64("h2d_ns") / 1000);
  if (name == "d2hTimeUs") return (unsigned int)(stat64("d2h_ns") / 1000);
  if (name == "algKBytes") return (unsigned int)(stat64(regs()->beta ? "alg_bytes_beta1" : "alg_bytes") / 1024);
  if (name == "mode") return regs()->mode;
  if (name == "kernel") return (unsigned int)stat64("kernel");
  if (name == "device") return regs()->device;
  if (name == "error") return (unsigned int)m_status;
  return HardwareSpMV::statInt(name);
}

HardwareSpMV* makeHIPSpMVRef(unsigned int aBase, unsigned int aReset, SparseMatrix* A, SpMVData* x, SpMVData* y) {
  const unsigned int sign = *(volatile unsigned int*)(uintptr_t)aBase;  // as HWSpMVFactory.cpp:22
  if (sign == HIPSpMVRef::expSignature()) return new HIPSpMVRef(aBase, aReset, A, x, y);
  return 0;
}

std::string nameHIPSpMVRef(unsigned int aBase) {
  const unsigned int sign = *(volatile unsigned int*)(uintptr_t)aBase;
  return sign == HIPSpMVRef::expSignature() ? "HIPSpMV" : "";
}
