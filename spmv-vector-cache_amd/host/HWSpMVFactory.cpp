#include "HWSpMVFactory.h"

#include <iostream>

#include "HIPSpMV.h"

HWSpMVFactory::HWSpMVFactory() {}
HWSpMVFactory::~HWSpMVFactory() {}

static uint32_t readSignature(uintptr_t aBase) {
  return aBase ? *reinterpret_cast<volatile const uint32_t*>(aBase) : 0u;
}

// Dispatch on the 32-bit signature at aBase (HWSpMVFactory.cpp:20-38).  The
// reference asserts on an unknown signature; here the caller gets nullptr.
HardwareSpMV* HWSpMVFactory::make(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y) {
  const uint32_t sign = readSignature(aBase);
  if (sign == HIPSpMV::expSignature()) return new HIPSpMV(aBase, aReset, A, x, y);
  std::cout << "Accelerator signature unrecognized! " << std::hex << sign << std::dec << std::endl;
  return nullptr;
}

std::string HWSpMVFactory::name(uintptr_t aBase) {
  const uint32_t sign = readSignature(aBase);
  if (sign == HIPSpMV::expSignature()) return "HIPSpMV";
  std::cout << "Accelerator signature unrecognized! " << std::hex << sign << std::dec << std::endl;
  return "<undefined>";
}
