#include "HardwareSpMV.h"

#include <cstring>

// software/HardwareSpMV.cpp:8-25.  The reference asserts 64-byte alignment of
// every buffer because its DMA engines burst on 64-byte lines; the HIP backend
// stages host buffers through its own device copies, so alignment is not
// required here.  Thresholds default to 128 like the reference.
HardwareSpMV::HardwareSpMV(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y)
    : SpMV(A, x, y),
      m_accelBase(reinterpret_cast<volatile uint32_t*>(aBase)),
      m_resetBase(reinterpret_cast<volatile uint32_t*>(aReset)) {}

HardwareSpMV::~HardwareSpMV() {}

// Pulse the reset word (HardwareSpMV.cpp:31-35); the result is "not compared
// yet" until compareGolden runs.
void HardwareSpMV::resetAccelerator() {
  if (m_resetBase) {
    *m_resetBase = 1;
    *m_resetBase = 0;
  }
  m_diffFromGolden = 1;
}

void HardwareSpMV::compareGolden(SpMVData* golden) {
  m_diffFromGolden = std::memcmp(golden, m_y, sizeof(SpMVData) * m_A->getRows());
}

unsigned int HardwareSpMV::statInt(std::string name) {
  if (name == "diffFromGolden") return (unsigned int)m_diffFromGolden;
  if (name == "rows") return m_A->getRows();
  if (name == "cols") return m_A->getCols();
  if (name == "nz") return m_A->getNz();
  return 0;
}

std::vector<std::string> HardwareSpMV::statKeys() { return {"diffFromGolden", "rows", "cols", "nz"}; }

void HardwareSpMV::init() {}
void HardwareSpMV::write() {}
void HardwareSpMV::regular() {}

void HardwareSpMV::setThresholds(unsigned int colPtr, unsigned int rowInd, unsigned int nzData, unsigned int inpVec) {
  m_thres = Thresholds{colPtr, rowInd, nzData, inpVec};
}

void HardwareSpMV::setupRegs() { setThresholdRegisters(); }
