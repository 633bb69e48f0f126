// Internal declarations shared by the libhipspmv.so translation units.
// Not part of the ABI (include/hipspmv.h is).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace hipspmv {

// ---- vcache kernel geometry ---------------------------
// One 1024-thread workgroup per row block; LDS holds the block's y accumulators
// (<= kVcRows doubles), two x panels of kVcPanel doubles and the block's
// segment table (<= kVcSegMax offsets): 32768 + 130048 + 1024 = 163840 B.
constexpr int kVcThreads = 1024;
constexpr int kVcRows = 4096;
constexpr int kVcPanel = 8128;
constexpr int kVcSegMax = 256;        // npad + 1 <= kVcSegMax
constexpr int kVcEpt = 2;             // entries per thread held in registers per panel
constexpr int kVcDepth = 2;           // panels of prefetch in flight (entries + x)
constexpr uint32_t kVcCont = 1u << 30;  // entry continues the previous entry's row run
constexpr uint32_t kVcMore = 1u << 31;  // next entry continues this entry's row run

// ---- csr_vector geometry ---------------------------------------------------
constexpr int kCvGroupNnz = 256;  // max nnz of a multi-row group (4 per lane)
constexpr int kCvGroupRows = 64;  // max rows of a multi-row group (1 per lane)

struct HostCSR {
  uint32_t rows = 0, cols = 0, nnz = 0;
  std::vector<uint32_t> rowptr, colind;
  std::vector<uint64_t> vals;  // 8-byte words (f64 bits or u64)
};

struct VcacheLayout {
  uint32_t rows_per_block = 0, nblocks = 0, npanels = 0, npad = 0;
  std::vector<uint32_t> seg;    // nblocks * (npad + 1) global entry offsets
  std::vector<uint32_t> code;   // per entry: col_local | row_local << 16 | CONT | MORE
  std::vector<uint64_t> vals;   // per entry
  uint32_t max_seg = 0;
};

// CSC (SparseMatrix layout) -> CSR, stable, masking bits 30-31 of the row ids.
// Returns a HIPSPMV_* status; fills `why` on validation failure.
int csc_to_csr(const uint32_t* colptr, const uint32_t* rowind, const void* vals, uint32_t rows, uint32_t cols,
               uint32_t nnz, HostCSR& out, std::string& why);
int copy_csr(const uint32_t* rowptr, const uint32_t* colind, const void* vals, uint32_t rows, uint32_t cols,
             uint32_t nnz, HostCSR& out, std::string& why);

bool vcache_eligible(const HostCSR& a);
void build_vcache(const HostCSR& a, VcacheLayout& out);
// Row groups for csr_vector: group g covers rows [groups[g], groups[g+1]).
void build_row_groups(const HostCSR& a, std::vector<uint32_t>& groups);

}  // namespace hipspmv
