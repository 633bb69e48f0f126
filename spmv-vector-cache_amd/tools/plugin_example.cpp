// plugin_example: the INTEGRATION.md section A program, compiled and run by the
// GPU tests so the documented drop-in path stays true.
//
// Loads a reference-format matrix, computes the SoftwareSpMV golden, then the
// same product through HWSpMVFactory -> HIPSpMV (the reference's
// software/main.cpp:225-247 sequence), on one device and on N devices of this
// process, and prints diffFromGolden for each.
//   plugin_example <dir> <name> [ndev]
#include <cstdlib>
#include <iostream>
#include <vector>

#include "HIPSpMV.h"
#include "HWSpMVFactory.h"
#include "MatrixIO.h"
#include "SoftwareSpMV.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: plugin_example <dir> <name> [ndev]" << std::endl;
    return 2;
  }
  const int ndev = argc > 3 ? std::atoi(argv[3]) : 1;
  SparseMatrix* A = loadSparseMatrix(argv[1], argv[2]);
  if (!A) return 2;
  std::vector<SpMVData> x(A->getCols(), 1.0), y(A->getRows(), 0.0);
  SoftwareSpMV golden(A, x.data());  // main.cpp:225-226
  golden.exec();

  // The register block replaces accBase/resBase (main.cpp:18-19).
  HIPSpMVRegisterFile* regs = HIPSpMV::registerFile(0);
  regs->mode = HIPSPMV_MODE_ORDERED;  // bit-identical to SoftwareSpMV
  regs->beta = 1;                     // y += A*x, as SoftwareSpMV
  int visible = 1;
  if (hipspmv_device_count(&visible) != HIPSPMV_OK || visible < 1) visible = 1;
  int failures = 0;
  for (int n : {1, ndev}) {
    regs->num_devices = n;  // > 1: rows split over devices, x broadcast device to device
    for (int d = 0; d < n; ++d) regs->devices[d] = d % visible;
    const uintptr_t accBase = reinterpret_cast<uintptr_t>(regs);
    const uintptr_t resBase = reinterpret_cast<uintptr_t>(&regs->reset);
    HardwareSpMV* spmv = HWSpMVFactory::make(accBase, resBase, A, x.data(), y.data());
    if (!spmv) return 2;
    std::fill(y.begin(), y.end(), 0.0);
    const bool ok = spmv->exec();
    spmv->compareGolden(golden.getY());
    std::cout << HWSpMVFactory::name(accBase) << " devices=" << spmv->statInt("numDevices")
              << " exec=" << ok << " diffFromGolden=" << spmv->statInt("diffFromGolden")
              << " kernelTimeUs=" << spmv->statInt("kernelTimeUs") << std::endl;
    failures += !ok || spmv->statInt("diffFromGolden") != 0;
    delete spmv;
  }
  delete A;
  return failures ? 1 : 0;
}
