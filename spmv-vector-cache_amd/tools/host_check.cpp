// host_check: drives the host plugin surface (host/*.cpp) on the reference
// fixtures with no GPU, for sanitizer builds (tests/test_host_sanitize.py
// compiles it with -fsanitize=address,undefined).  Exit 0 = every check
// passed; the sanitizers abort on the first memory or UB error.
//
//   host_check <matrices dir> <tmp dir> <fixture>...
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include <sys/stat.h>

#include "MatrixIO.h"
#include "MatrixOps.h"
#include "SoftwareSpMV.h"
#include "SparseMatrix.h"
#include "Synthetic.h"
#include "csr2csc.h"

static int g_fail = 0;
#define CHECK(cond)                                                           \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
      ++g_fail;                                                               \
    }                                                                         \
  } while (0)

static bool file_exists(const std::string& p) { return std::ifstream(p).good(); }

static std::vector<SpMVData> sw_exec(SparseMatrix* A, const std::vector<SpMVData>* x = nullptr) {
  std::vector<SpMVData> y(A->getRows(), 0.0);
  std::vector<SpMVData> xv = x ? *x : std::vector<SpMVData>();
  SoftwareSpMV sw(A, x ? xv.data() : nullptr, y.data());
  CHECK(sw.exec());
  return y;
}

static void check_fixture(const std::string& dir, const std::string& tmp, const std::string& name) {
  SparseMatrix* A = loadSparseMatrix(dir, name);
  CHECK(A != nullptr);
  if (!A) return;
  const unsigned rows = A->getRows(), cols = A->getCols(), nz = A->getNz();
  std::vector<SpMVData> y = sw_exec(A);
  // compareGolden (HardwareSpMV.cpp:37-39): the reference's own golden.bin
  const std::string gpath = dir + "/" + name + "/golden.bin";
  if (A->getDataType() == SPMV_F64 && file_exists(gpath)) {
    std::vector<SpMVData> g(rows);
    CHECK(loadGolden(gpath, rows, g.data()));
    CHECK(std::memcmp(g.data(), y.data(), 8ull * rows) == 0);
  }
  // preprocessing statistics leave the matrix unmarked (SoftwareSpMV.cpp:72-95)
  std::vector<SpMVIndex> inds(A->getInds(), A->getInds() + nz);
  {
    SoftwareSpMV sw(A);
    sw.measurePreprocessingTimes();
    CHECK(sw.statInt("maxAlive") <= rows);
    CHECK(std::memcmp(inds.data(), A->getInds(), 4ull * nz) == 0);
    CHECK(sw.statKeys().size() == 9);
  }
  A->markRowStarts(true, 30);
  A->clearRowMarkings(~(1u << 30));
  CHECK(std::memcmp(inds.data(), A->getInds(), 4ull * nz) == 0);
  // CSC -> CSR -> CSC is the identity (stable counting sort both ways)
  {
    std::vector<uint64_t> a(nz), at(nz), att(nz);
    std::memcpy(a.data(), A->getNzData(), 8ull * nz);
    std::vector<uint32_t> ri(nz), rs(rows + 1), ci(nz), cs(cols + 1);
    csr2csc(cols, rows, nz, a.data(), A->getInds(), A->getIndPtrs(), at.data(), ri.data(), rs.data());
    csr2csc(rows, cols, nz, at.data(), ri.data(), rs.data(), att.data(), ci.data(), cs.data());
    CHECK(std::memcmp(cs.data(), A->getIndPtrs(), 4ull * (cols + 1)) == 0);
    CHECK(std::memcmp(ci.data(), A->getInds(), 4ull * nz) == 0);
    CHECK(std::memcmp(att.data(), a.data(), 8ull * nz) == 0);
  }
  // row-length histogram and the longest-row-first permutation (matrixutils.py:116-158)
  {
    auto hist = rowLenHistogram(A);
    uint64_t total = 0;
    for (auto& kv : hist) total += kv.second;
    CHECK(total <= rows);
    auto perm = longestRowFirstPermutation(A);
    CHECK(perm.size() == rows);
    std::vector<char> seen(rows, 0);
    for (uint32_t p : perm)
      if (p < rows) seen[p] = 1;
    for (char s : seen) CHECK(s);
    SparseMatrix* P = permuteRows(A, perm);
    CHECK(P && P->getNz() == nz);
    if (P) {
      std::vector<SpMVData> yp = sw_exec(P);
      // row i of P is row perm[i] of A
      for (unsigned i = 0; i < rows; ++i) CHECK(std::memcmp(&yp[i], &y[perm[i]], 8) == 0);
      delete P;
    }
  }
  // .bin writer round trip
  {
    const std::string out = tmp + "/rt";
    ::mkdir(out.c_str(), 0755);
    ::mkdir((out + "/" + name).c_str(), 0755);
    CHECK(writeSparseMatrix(A, out, name));
    SparseMatrix* B = loadSparseMatrix(out, name);
    CHECK(B && B->getRows() == rows && B->getCols() == cols && B->getNz() == nz);
    if (B) {
      CHECK(std::memcmp(B->getIndPtrs(), A->getIndPtrs(), 4ull * (cols + 1)) == 0);
      CHECK(std::memcmp(B->getInds(), A->getInds(), 4ull * nz) == 0);
      CHECK(std::memcmp(B->getNzData(), A->getNzData(), 8ull * nz) == 0);
      delete B;
    }
  }
  delete A;
}

static void check_synthetic() {
  // stripe generator: rows of a range equal the same rows of the whole
  const uint32_t n = 4096, k = 32;
  std::vector<uint32_t> rp(n + 1), ci(n * k);
  std::vector<double> v(n * k);
  genStripeCSR(0, n, n, k, 1, 2, rp.data(), ci.data(), v.data());
  std::vector<uint32_t> rp2(1001), ci2(1000 * k);
  std::vector<double> v2(1000 * k);
  genStripeCSR(1234, 1000, n, k, 1, 2, rp2.data(), ci2.data(), v2.data());
  CHECK(std::memcmp(ci2.data(), ci.data() + 1234 * k, 4ull * 1000 * k) == 0);
  CHECK(std::memcmp(v2.data(), v.data() + 1234 * k, 8ull * 1000 * k) == 0);
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t j = rp[r] + 1; j < rp[r + 1]; ++j) CHECK(ci[j - 1] < ci[j]);
  // R-MAT: row ranges concatenate to the whole matrix; partitions cover all rows
  const uint32_t scale = 10;
  std::vector<uint32_t> rpa, cia, rpb, cib, rpc, cic;
  std::vector<double> va, vb, vc;
  const uint64_t nnz = genRmatCSR(scale, 16, 4, 0.57, 0.19, 0.19, rpa, cia, va);
  const uint32_t mid = 300;
  const uint64_t n1 = genRmatCSRRows(scale, 16, 4, 0.57, 0.19, 0.19, 0, mid, rpb, cib, vb);
  const uint64_t n2 = genRmatCSRRows(scale, 16, 4, 0.57, 0.19, 0.19, mid, 1u << scale, rpc, cic, vc);
  CHECK(n1 + n2 == nnz);
  CHECK(std::memcmp(cib.data(), cia.data(), 4ull * n1) == 0);
  CHECK(std::memcmp(cic.data(), cia.data() + n1, 4ull * n2) == 0);
  std::vector<uint32_t> counts(1u << scale), b1(9), b2(9);
  genRmatRowCounts(scale, 16, 4, 0.57, 0.19, 0.19, counts.data());
  partitionRowCounts(counts.data(), 1u << scale, 8, b1.data());
  partitionRows(rpa.data(), 1u << scale, 8, b2.data());
  CHECK(b1[0] == 0 && b1[8] == (1u << scale) && b2[0] == 0 && b2[8] == (1u << scale));
  for (int i = 0; i < 8; ++i) CHECK(b1[i] <= b1[i + 1] && b2[i] <= b2[i + 1]);
  // degenerate partitions: more parts than rows
  std::vector<uint32_t> b3(65);
  partitionRows(rpa.data(), 3, 64, b3.data());
  CHECK(b3[64] == 3);
}

static void check_mtx(const std::string& dir, const std::string& tmp) {
  const std::string mtx = dir + "/mtx/circuit204.mtx";
  if (!file_exists(mtx)) return;
  SparseMatrix* M = loadMatrixMarket(mtx);
  CHECK(M != nullptr);
  if (!M) return;
  SparseMatrix* R = loadSparseMatrix(dir, "circuit204");
  CHECK(R && R->getNz() == M->getNz());
  if (R && R->getNz() == M->getNz()) {
    CHECK(std::memcmp(R->getInds(), M->getInds(), 4ull * R->getNz()) == 0);
    CHECK(std::memcmp(R->getNzData(), M->getNzData(), 8ull * R->getNz()) == 0);
  }
  CHECK(writeGolden(M, tmp + "/golden.bin"));
  delete R;
  delete M;
  // malformed inputs are refused, not crashed on
  const std::string bad = tmp + "/bad.mtx";
  {
    std::ofstream f(bad);
    f << "%%MatrixMarket matrix coordinate real general\n3 3 2\n1 1 1.0\n9 9 2.0\n";
  }
  SparseMatrix* B = loadMatrixMarket(bad);
  CHECK(B == nullptr);
  delete B;
  {
    std::ofstream f(bad);
    f << "%%MatrixMarket matrix coordinate real general\n3 3 5\n1 1 1.0\n";
  }
  B = loadMatrixMarket(bad);
  CHECK(B == nullptr);
  delete B;
  CHECK(loadSparseMatrix(tmp, "does-not-exist") == nullptr);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: host_check <matrices dir> <tmp dir> <fixture>...\n");
    return 2;
  }
  const std::string dir = argv[1], tmp = argv[2];
  for (int i = 3; i < argc; ++i) check_fixture(dir, tmp, argv[i]);
  check_synthetic();
  check_mtx(dir, tmp);
  std::printf("host_check: %d failures\n", g_fail);
  return g_fail ? 1 : 0;
}
