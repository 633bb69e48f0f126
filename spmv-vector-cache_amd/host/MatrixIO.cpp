#include "MatrixIO.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <vector>

#include "SoftwareSpMV.h"

namespace {

bool readFile(const std::string& path, std::vector<char>& buf) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return true;
}

bool writeFile(const std::string& path, const void* data, size_t bytes) {
  std::ofstream f(path, std::ios::binary);
  if (!f) return false;
  f.write(static_cast<const char*>(data), (std::streamsize)bytes);
  return (bool)f;
}

template <typename T>
T* copyOut(const std::vector<char>& buf, size_t count) {
  T* p = new T[count ? count : 1];
  if (count) std::memcpy(p, buf.data(), sizeof(T) * count);
  return p;
}

uint32_t alignedIncrement(uint32_t base, uint32_t inc, uint32_t align) {  // matrixutils.py:174-180
  uint32_t r = base + inc;
  if (r % align) r += align - r % align;
  return r;
}

}  // namespace

SparseMatrix* loadSparseMatrix(const std::string& dir, const std::string& name) {
  const std::string base = dir + "/" + name + "/" + name;
  std::vector<char> meta, ptr, ind, dat;
  if (!readFile(base + "-meta.bin", meta) || meta.size() < sizeof(CompressedSparseMetadata)) {
    std::cerr << "loadSparseMatrix: cannot read " << base << "-meta.bin" << std::endl;
    return nullptr;
  }
  CompressedSparseMetadata md;
  std::memcpy(&md, meta.data(), sizeof md);
  if (!readFile(base + "-indptr.bin", ptr) || !readFile(base + "-inds.bin", ind) ||
      !readFile(base + "-data.bin", dat)) {
    std::cerr << "loadSparseMatrix: missing files for " << base << std::endl;
    return nullptr;
  }
  if (ptr.size() != 4ull * (md.numCols + 1ull) || ind.size() != 4ull * md.numNZ || dat.size() != 8ull * md.numNZ) {
    std::cerr << "loadSparseMatrix: file sizes disagree with metadata for " << base << std::endl;
    return nullptr;
  }
  SparseMatrix* A = SparseMatrix::fromArrays(
      md.numRows, md.numCols, md.numNZ, copyOut<SpMVIndex>(ptr, md.numCols + 1ull), copyOut<SpMVIndex>(ind, md.numNZ),
      copyOut<SpMVData>(dat, md.numNZ), name.find("uint64") != std::string::npos ? SPMV_U64 : SPMV_F64, true);
  A->setName(name);
  return A;
}

bool loadGolden(const std::string& path, unsigned int rows, SpMVData* out) {
  std::vector<char> buf;
  if (!readFile(path, buf) || buf.size() != 8ull * rows) return false;
  std::memcpy(out, buf.data(), buf.size());
  return true;
}

SparseMatrix* loadMatrixMarket(const std::string& path) {
  std::ifstream f(path);
  if (!f) return nullptr;
  std::string line;
  if (!std::getline(f, line)) return nullptr;
  std::string banner = line;
  std::transform(banner.begin(), banner.end(), banner.begin(), ::tolower);
  if (banner.rfind("%%matrixmarket matrix coordinate", 0) != 0) {
    std::cerr << "loadMatrixMarket: only coordinate matrices are supported" << std::endl;
    return nullptr;
  }
  const bool pattern = banner.find(" pattern") != std::string::npos;
  const bool symmetric = banner.find(" symmetric") != std::string::npos;
  const bool skew = banner.find(" skew-symmetric") != std::string::npos;
  const bool integer = banner.find(" integer") != std::string::npos;
  while (std::getline(f, line))
    if (!line.empty() && line[0] != '%') break;
  unsigned long rows = 0, cols = 0, entries = 0;
  if (std::sscanf(line.c_str(), "%lu %lu %lu", &rows, &cols, &entries) != 3) return nullptr;
  struct Trip { uint32_t r, c; double v; uint64_t order; };
  std::vector<Trip> t;
  t.reserve(entries * (symmetric || skew ? 2 : 1));
  for (unsigned long i = 0; i < entries; ++i) {
    unsigned long r, c;
    double v = 1.0;
    if (!(f >> r >> c)) return nullptr;
    if (!pattern && !(f >> v)) return nullptr;
    if (r < 1 || r > rows || c < 1 || c > cols) return nullptr;
    t.push_back({(uint32_t)(r - 1), (uint32_t)(c - 1), v, t.size()});
    if ((symmetric || skew) && r != c) t.push_back({(uint32_t)(c - 1), (uint32_t)(r - 1), skew ? -v : v, t.size()});
  }
  (void)integer;
  // column-major, rows ascending, duplicates summed in file order
  std::stable_sort(t.begin(), t.end(), [](const Trip& a, const Trip& b) { return a.c != b.c ? a.c < b.c : a.r < b.r; });
  std::vector<uint32_t> ptr(cols + 1, 0), ind;
  std::vector<double> val;
  for (size_t i = 0; i < t.size(); ++i) {
    if (!ind.empty() && i > 0 && t[i].c == t[i - 1].c && t[i].r == t[i - 1].r) {
      val.back() += t[i].v;
      continue;
    }
    ind.push_back(t[i].r);
    val.push_back(t[i].v);
    ptr[t[i].c + 1]++;
  }
  for (unsigned long c = 0; c < cols; ++c) ptr[c + 1] += ptr[c];
  SpMVIndex* P = new SpMVIndex[cols + 1];
  SpMVIndex* I = new SpMVIndex[ind.size() ? ind.size() : 1];
  SpMVData* V = new SpMVData[val.size() ? val.size() : 1];
  std::copy(ptr.begin(), ptr.end(), P);
  std::copy(ind.begin(), ind.end(), I);
  std::copy(val.begin(), val.end(), V);
  SparseMatrix* A = SparseMatrix::fromArrays((unsigned)rows, (unsigned)cols, (unsigned)ind.size(), P, I, V, SPMV_F64,
                                             true);
  const size_t slash = path.find_last_of('/');
  std::string nm = path.substr(slash == std::string::npos ? 0 : slash + 1);
  if (nm.size() > 4 && nm.compare(nm.size() - 4, 4, ".mtx") == 0) nm.resize(nm.size() - 4);
  A->setName(nm);
  return A;
}

bool writeSparseMatrix(const SparseMatrix* A, const std::string& dir, const std::string& name) {
  const std::string base = dir + "/" + name + "/" + name;
  const uint32_t ptrBytes = 4u * (A->getCols() + 1), indBytes = 4u * A->getNz();
  CompressedSparseMetadata md;
  md.numRows = A->getRows();
  md.numCols = A->getCols();
  md.numNZ = A->getNz();
  md.startingRow = 0;
  md.indPtrBase = alignedIncrement(0x8000100u, 28, 64);
  md.indBase = alignedIncrement(md.indPtrBase, ptrBytes, 64);
  md.nzDataBase = alignedIncrement(md.indBase, indBytes, 64);
  return writeFile(base + "-meta.bin", &md, sizeof md) && writeFile(base + "-indptr.bin", A->getIndPtrs(), ptrBytes) &&
         writeFile(base + "-inds.bin", A->getInds(), indBytes) &&
         writeFile(base + "-data.bin", A->getNzData(), 8ull * A->getNz());
}

bool writeGolden(const SparseMatrix* A, const std::string& path) {
  SoftwareSpMV sw(const_cast<SparseMatrix*>(A));
  sw.exec();
  return writeFile(path, sw.getY(), 8ull * A->getRows());
}
