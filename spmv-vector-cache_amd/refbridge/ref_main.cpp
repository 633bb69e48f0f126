// refbridge: the reference's own benchmark pipeline (ref:software/main.cpp:
// 195-256) on the reference's own plugin classes -- SparseMatrix::fromMemory,
// SparseMatrix::markRowStarts, HardwareSpMV (compiled unmodified from
// /root/reference/software) -- with the HIP backend registered through the
// factory branch of HIPSpMVRef.h.  Demonstrates INTEGRATION.md section B as
// a built program; test infrastructure, built into oracle/_ref/ only where the
// reference tree exists (oracle/Makefile target `refbridge`).
//
// The reference runs on a 32-bit Zynq: SparseMatrix::fromMemory takes the
// 32-bit address of a CompressedSparseMetadata block whose fields are 32-bit
// addresses of the arrays (SparseMatrix.cpp:29-50), and HardwareSpMV takes
// 32-bit register addresses (HardwareSpMV.h:10-11).  On x86-64 the matrix
// files and the register block are therefore placed below 2 GiB with
// mmap(MAP_32BIT), where the SD-card loader (main.cpp:26-37) placed them in
// the Zynq's DDR; x and y come from the reference's malloc_aligned, as in
// main.cpp:210-215.  The hardware result is compared with golden.bin (A*1,
// the value SoftwareSpMV computes for x = 1, y = 0: tests/test_oracle.py)
// through the reference's HardwareSpMV::compareGolden.
//
//   refbridge --dir D [--cms 0|1] [--mode ordered|fast] [--kernel K] [--device N] [--reps R] names...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <iostream>
#include <string>
#include <vector>

#include "HIPSpMVRef.h"
#include "SparseMatrix.h"  // the reference's
#include "malloc_aligned.h"

namespace {

struct Arena {  // one MAP_32BIT mapping, bump-allocated in 64-byte steps
  char* base = 0;
  size_t size = 0, used = 0;
  bool map(size_t bytes) {
    size = (bytes + 4095) & ~(size_t)4095;
    void* p = mmap(0, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
    if (p == MAP_FAILED) return false;
    base = (char*)p;
    used = 0;
    return (uintptr_t)base + size <= 0xFFFFFFFFull;
  }
  void* take(size_t bytes) {
    void* p = base + used;
    used += (bytes + 63) & ~(size_t)63;
    return used <= size ? p : 0;
  }
  ~Arena() {
    if (base) munmap(base, size);
  }
};

long file_size(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fclose(f);
  return n;
}

bool read_into(const std::string& path, void* dst, size_t bytes) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  const size_t got = fread(dst, 1, bytes, f);
  fclose(f);
  return got == bytes;
}

unsigned int addr32(const void* p) { return (unsigned int)(uintptr_t)p; }

}  // namespace

int main(int argc, char** argv) {
  std::string dir = ".";
  int cms = 0, mode = HIPSPMV_MODE_ORDERED, kernel = HIPSPMV_KERNEL_AUTO, device = 0, reps = 1;
  std::vector<std::string> names;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--dir" && i + 1 < argc) dir = argv[++i];
    else if (a == "--cms" && i + 1 < argc) cms = atoi(argv[++i]);
    else if (a == "--mode" && i + 1 < argc) mode = std::string(argv[++i]) == "fast" ? HIPSPMV_MODE_FAST : HIPSPMV_MODE_ORDERED;
    else if (a == "--kernel" && i + 1 < argc) kernel = atoi(argv[++i]);
    else if (a == "--device" && i + 1 < argc) device = atoi(argv[++i]);
    else if (a == "--reps" && i + 1 < argc) reps = atoi(argv[++i]);
    else names.push_back(a);
  }

  // the register block and its reset word, below 4 GiB (main.cpp:18-19 fixed them at 0x40000000 / 0x43c00000)
  Arena regs_arena;
  if (!regs_arena.map(4096)) {
    std::cerr << "refbridge: MAP_32BIT mapping failed" << std::endl;
    return 2;
  }
  HIPSpMVRefRegs* regs = (HIPSpMVRefRegs*)regs_arena.take(sizeof(HIPSpMVRefRegs));
  volatile uint32_t* reset = (volatile uint32_t*)regs_arena.take(64);
  regs->signature = HIPSpMVRef::expSignature();
  regs->device = (uint32_t)device;
  regs->mode = (uint32_t)mode;
  regs->kernel = (uint32_t)kernel;
  regs->beta = 1;  // y += A*x, the reference's semantics (SoftwareSpMV.cpp:62)
  regs->dtype = HIPSPMV_F64;
  *reset = 0;
  const unsigned int accBase = addr32(regs), resBase = addr32((const void*)reset);

  bool keysBuilt = false;
  std::vector<std::string> keys;
  int failures = 0;
  for (size_t m = 0; m < names.size(); ++m) {
    const std::string& name = names[m];
    const std::string base = dir + "/" + name + "/" + name;
    const long szp = file_size(base + "-indptr.bin"), szi = file_size(base + "-inds.bin"),
               szd = file_size(base + "-data.bin"), szg = file_size(dir + "/" + name + "/golden.bin");
    if (szp < 0 || szi < 0 || szd < 0 || szg < 0) {
      std::cerr << "refbridge: " << name << ": missing files (indptr/inds/data/golden.bin)" << std::endl;
      return 2;
    }
    // the SD-card loader, relocated: metadata + arrays in one low mapping
    Arena mat;
    if (!mat.map(sizeof(CompressedSparseMetadata) + szp + szi + szd + 4 * 64)) {
      std::cerr << "refbridge: MAP_32BIT mapping failed" << std::endl;
      return 2;
    }
    CompressedSparseMetadata* md = (CompressedSparseMetadata*)mat.take(sizeof(CompressedSparseMetadata));
    if (!read_into(base + "-meta.bin", md, sizeof(*md))) {
      std::cerr << "refbridge: " << name << ": bad -meta.bin" << std::endl;
      return 2;
    }
    void* indptr = mat.take(szp);
    void* inds = mat.take(szi);
    void* data = mat.take(szd);
    if (!read_into(base + "-indptr.bin", indptr, szp) || !read_into(base + "-inds.bin", inds, szi) ||
        !read_into(base + "-data.bin", data, szd)) {
      std::cerr << "refbridge: " << name << ": short read" << std::endl;
      return 2;
    }
    md->indPtrBase = addr32(indptr);
    md->indBase = addr32(inds);
    md->nzDataBase = addr32(data);

    SparseMatrix* A = SparseMatrix::fromMemory(addr32(md));  // the reference's loader
    if (!A) return 2;
    A->setName(name);
    SpMVData* x = (SpMVData*)malloc_aligned(64, sizeof(SpMVData) * A->getCols());
    SpMVData* y = (SpMVData*)malloc_aligned(64, sizeof(SpMVData) * A->getRows());
    SpMVData* golden = (SpMVData*)malloc_aligned(64, sizeof(SpMVData) * A->getRows());
    if ((long)(sizeof(SpMVData) * A->getRows()) != szg || !read_into(dir + "/" + name + "/golden.bin", golden, szg)) {
      std::cerr << "refbridge: " << name << ": golden.bin does not match the row count" << std::endl;
      return 2;
    }
    for (SpMVIndex i = 0; i < A->getCols(); i++) x[i] = (SpMVData)1;  // main.cpp:217-222

    if (cms) A->markRowStarts();  // main.cpp:228-229, the reference's own marking

    HardwareSpMV* spmv = makeHIPSpMVRef(accBase, resBase, A, x, y);
    if (!spmv) {
      std::cerr << "refbridge: signature unrecognised" << std::endl;
      return 2;
    }
    if (!keysBuilt) {  // main.cpp:239-246
      keys = spmv->statKeys();
      keys.push_back("accType");
      keys.push_back("matrix");
      for (size_t k = 0; k < keys.size(); ++k) std::cout << keys[k] << ",";
      std::cout << std::endl;
      keysBuilt = true;
    }
    for (int r = 0; r < reps; ++r) {
      for (SpMVIndex i = 0; i < A->getRows(); i++) y[i] = (SpMVData)0;
      if (!spmv->exec()) ++failures;
    }
    spmv->compareGolden(golden);  // main.cpp:250, the reference's memcmp
    for (size_t k = 0; k < keys.size(); ++k) {  // main.cpp:56-66
      if (keys[k] == "matrix")
        std::cout << name << ",";
      else if (keys[k] == "accType")
        std::cout << nameHIPSpMVRef(accBase) << ",";
      else
        std::cout << spmv->statInt(keys[k]) << ",";
    }
    std::cout << std::endl;
    delete spmv;
    free_aligned(x);
    free_aligned(y);
    free_aligned(golden);
    delete A;
  }
  return failures ? 1 : 0;
}
