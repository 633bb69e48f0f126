// spmvbench: the benchmark driver of software/main.cpp:146-264, on MI355X.
//
// Same protocol: a list of configurations, the cold-miss-skip flag and a list
// of matrices, read from stdin ("q" ends each list) unless given on the
// command line.  For every (configuration, matrix): load the matrix
// (main.cpp:26-37), x = 1 and y = 0 (:210-222), SoftwareSpMV golden
// (:225-226), optional CMS marking (:228-229), HWSpMVFactory::make, exec,
// compareGolden, one CSV row of statKeys() + accType + matrix (:49-66).
// Configurations: "hip" (HIPSpMV on the device of --device), "hip<N>"
// (HIPSpMV row-partitioned over N devices of this process, ids wrapping
// around the visible devices) and "sw" (benchmarkSW, :102-144).  Times are
// microseconds.
//
//   spmvbench [--dir D] [--device N] [--mode ordered|fast] [--kernel K] [--reps N]
//             [--cms 0|1] [--confs hip,sw] [--profile 0|1] matrix...
// --profile 1: vcache-family launches record the NewCache state statistics
// (sActive ... noReadyButValid), measured in-kernel.
// --pmc FILE: a rocprofv3 --pmc counter CSV of the backend's kernel; readMisses,
// hazardStalls and capacityStalls report its counters (HIPSpMV::setPmcCsv).
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "HIPSpMV.h"
#include "HWSpMVFactory.h"
#include "MatrixIO.h"
#include "SoftwareSpMV.h"
#include "hipspmv.h"

namespace {

std::string g_loaded;

void printKeys(const std::vector<std::string>& keys) {
  for (const auto& k : keys) std::cout << k << ",";
  std::cout << std::endl;
}

void printResults(SpMV* spmv, const std::vector<std::string>& keys, uintptr_t accBase) {
  for (const auto& k : keys) {
    if (k == "matrix") std::cout << g_loaded << ",";
    else if (k == "accType") std::cout << HWSpMVFactory::name(accBase) << ",";
    else std::cout << spmv->statInt(k) << ",";
  }
  std::cout << std::endl;
}

void fillOnes(SparseMatrix* A, SpMVData* x) {
  for (unsigned i = 0; i < A->getCols(); ++i) {
    if (A->getDataType() == SPMV_U64) {
      const uint64_t one = 1;
      std::memcpy(&x[i], &one, 8);
    } else {
      x[i] = 1.0;
    }
  }
}

void benchmarkSW(const std::string& dir, const std::vector<std::string>& ms) {
  bool keysBuilt = false;
  std::vector<std::string> keys;
  for (const auto& m : ms) {
    SparseMatrix* A = loadSparseMatrix(dir, m);
    if (!A) continue;
    g_loaded = m;
    std::vector<SpMVData> x(A->getCols()), y(A->getRows(), 0.0);
    fillOnes(A, x.data());
    SoftwareSpMV spmv(A, x.data(), y.data());
    if (!keysBuilt) {
      keys = spmv.statKeys();
      keys.push_back("matrix");
      printKeys(keys);
      keysBuilt = true;
    }
    spmv.exec();
    spmv.measurePreprocessingTimes();
    printResults(&spmv, keys, 0);
    delete A;
  }
}

std::vector<std::string> readList() {
  std::vector<std::string> out;
  std::string s;
  while (std::cin >> s && s != "q") out.push_back(s);
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  std::string dir = "tests/golden/matrices";
  int device = 0, mode = HIPSPMV_MODE_ORDERED, kernel = HIPSPMV_KERNEL_AUTO, reps = 1, profile = 0;
  std::string pmc;
  bool cms = false, haveCms = false;
  std::vector<std::string> confs, ms;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--dir") dir = next();
    else if (a == "--device") device = std::atoi(next().c_str());
    else if (a == "--mode") mode = next() == "fast" ? HIPSPMV_MODE_FAST : HIPSPMV_MODE_ORDERED;
    else if (a == "--kernel") {
      const std::string k = next();
      kernel = k == "vcache" ? HIPSPMV_KERNEL_VCACHE
               : k == "vcache_split" ? HIPSPMV_KERNEL_VCACHE_SPLIT
               : k == "csr_lane" ? HIPSPMV_KERNEL_CSR_LANE
               : k == "csr_vector" ? HIPSPMV_KERNEL_CSR_VECTOR
               : k == "sell" ? HIPSPMV_KERNEL_SELL
               : k == "vcache_split4" ? HIPSPMV_KERNEL_VCACHE_SPLIT4
               : k == "wcsr" ? HIPSPMV_KERNEL_WCSR : HIPSPMV_KERNEL_AUTO;
    } else if (a == "--reps") reps = std::atoi(next().c_str());
    else if (a == "--profile") profile = std::atoi(next().c_str());
    else if (a == "--pmc") pmc = next();
    else if (a == "--cms") { cms = std::atoi(next().c_str()) != 0; haveCms = true; }
    else if (a == "--confs") {
      std::stringstream ss(next());
      std::string c;
      while (std::getline(ss, c, ',')) confs.push_back(c);
    } else ms.push_back(a);
  }
  if (confs.empty()) {
    std::cout << "Enter list of configurations (hip, sw), q to finalize: " << std::endl;
    confs = readList();
  }
  if (!haveCms) {
    std::cout << "Cold miss skip (0 to disable, 1 to enable): " << std::endl;
    std::cin >> cms;
  }
  if (ms.empty()) {
    std::cout << "Enter list of matrices, q to finalize: " << std::endl;
    ms = readList();
  }
  std::cout << "Benchmarking " << confs.size() << "x" << ms.size() << " confs x matrices..." << std::endl;
  std::cout << "=============================================================" << std::endl;

  HIPSpMVRegisterFile* regs = HIPSpMV::registerFile(device);
  regs->mode = mode;
  regs->kernel = kernel;
  regs->beta = 1;  // y += A*x on a zeroed y, as main.cpp does
  regs->profile = profile;
  const uintptr_t accBase = reinterpret_cast<uintptr_t>(regs);
  const uintptr_t resBase = reinterpret_cast<uintptr_t>(&regs->reset);
  int failures = 0;
  bool keysBuilt = false;
  std::vector<std::string> keys;
  for (const auto& cf : confs) {
    if (cf == "sw") {
      benchmarkSW(dir, ms);
      break;
    }
    int ndev = 1;
    if (cf.rfind("hip", 0) != 0 || (cf.size() > 3 && (ndev = std::atoi(cf.c_str() + 3)) < 1) || ndev > 16) {
      std::cout << "unknown configuration " << cf << std::endl;
      continue;
    }
    int visible = 1;
    if (hipspmv_device_count(&visible) != HIPSPMV_OK || visible < 1) visible = 1;
    regs->num_devices = ndev;
    for (int d = 0; d < ndev; ++d) regs->devices[d] = (device + d) % visible;
    for (const auto& m : ms) {
      SparseMatrix* A = loadSparseMatrix(dir, m);
      if (!A) {
        ++failures;
        continue;
      }
      g_loaded = m;
      std::vector<SpMVData> x(A->getCols()), y(A->getRows(), 0.0);
      fillOnes(A, x.data());
      SoftwareSpMV check(A, x.data());
      check.exec();
      if (cms) A->markRowStarts();
      HardwareSpMV* spmv = HWSpMVFactory::make(accBase, resBase, A, x.data(), y.data());
      if (!spmv) return 2;
      if (!pmc.empty())
        if (auto* hip = dynamic_cast<HIPSpMV*>(spmv)) hip->setPmcCsv(pmc);
      if (!keysBuilt) {
        keys = spmv->statKeys();
        keys.push_back("accType");
        keys.push_back("matrix");
        printKeys(keys);
        keysBuilt = true;
      }
      for (int r = 0; r < reps; ++r) {
        std::fill(y.begin(), y.end(), 0.0);
        if (!spmv->exec()) ++failures;
      }
      spmv->compareGolden(check.getY());
      printResults(spmv, keys, accBase);
      if (mode == HIPSPMV_MODE_ORDERED && spmv->statInt("diffFromGolden") != 0) ++failures;
      delete spmv;
      delete A;
    }
  }
  std::cout << "=============================================================" << std::endl;
  std::cout << "Benchmarking complete" << std::endl;
  return failures ? 1 : 0;
}
