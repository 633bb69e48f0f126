// Internal declarations shared by the libhipspmv.so translation units.
// Not part of the ABI (include/hipspmv.h is).
#pragma once

#include <algorithm>
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "hipspmv.h"

namespace hipspmv {

// ---- vcache kernel geometry ---------------------------
// One 1024-thread workgroup per work unit = (row block, column part); LDS
// holds the block's y accumulators (<= rows doubles), two x panels of `panel`
// doubles and the unit's segment table (<= kVcSegMax offsets), 163840 B total:
//   ordered: 4096 rows, 1 part   : 32768 + 2*8128*8 + 1024
//   split  : 12352 rows, 3 parts : 98816 + 2*4000*8 + 1024
// The split geometry cuts the x bytes each CU streams to a third (each CU's
// L1->L2 request slots are the measured limit; 3 parts beat
// 2 and 4 on C3: 131.7 vs 146 and 139.5 us) and combines the column-part
// partials in fixed order (p0 + p1 + p2), so it is deterministic but not
// bit-identical: FAST mode.  12352 rows is the LDS budget; the layout sizes
// its blocks to fill the chip once (vcache_rows_per_block: ceil(2^20 / 85) =
// 12337 rows on C3, 85 blocks x 3 parts = 255 units).
struct VcGeom {
  int rows, panel, split;
  int colbits = 16;  // entry code: col_local | row_local << colbits | CONT | MORE
  int segmax = 256;  // segment offsets per unit the kernel's LDS table holds (npad + 1 <= segmax)
};
constexpr VcGeom kVcOrdered{4096, 8128, 1};
constexpr VcGeom kVcSplit{12352, 4000, 3};
//   split4 : 16384 rows, 4 parts: 131072 + 2*1984*8 + 1024 (experimental)
constexpr VcGeom kVcSplit4{16384, 1984, 4};
// ---- k_wgather: the same segment layout over column WINDOWS of 2^16 columns
// (512 KiB of x, L2-resident) with x gathered from global memory instead of
// staged in LDS -- for matrices whose x is too wide for LDS streaming to pay
// (C4/C5: 16M columns).  y block in LDS (<= 16384 rows, 14 bits), ORDERED.
// Round 4: 16384-row blocks over 2^16-column windows instead of 8192 over
// 2^17 -- twice the entries per x line in a segment, so more gathers of a
// wave share a line once the segment is sorted by line (sort_segments_by_line):
// full C4 3417 us (8192 rows) -> 3296 (sorted) -> 2870 (16384 rows, sorted),
// profiles/r04/logs/sweep_c4_*.log.  512 windows of 2^16 at 2^24 columns: the
// kernel's segment table holds 512 offsets (segmax).
constexpr VcGeom kWgWindow{16384, 1 << 16, 1, 16, 512};
// ---- k_wgather, two column parts (FAST; kernel "wgather_split", round 6):
// a matrix of at most 128 * 16384 rows (a 2^21-row C4 shard) gets 16384-row
// blocks -- twice the entries per x line in a segment of the one-part
// layout's 8192 -- and each block's windows are cut in two halves, so the
// 256 work units still fill the chip once.  Units of part 0 run on XCDs 0-3,
// part 1 on XCDs 4-7 (workgroup w lands on XCD w mod 8): each XCD's L2 pulls
// half of x through instead of all of it -- half the memory-side x traffic,
// though not faster than alternating the parts (the gain is
// the 16384-row blocks and the entry residency).  y = p0 + p1 in part order
// (owner combine, combine.h): deterministic, not bit-identical to ORDERED.
constexpr VcGeom kWgSplit{16384, 1 << 16, 2, 16, 512};
// kWgSplit entry residency: the leading row blocks whose entries fit in
// kWgSplitMallBytes - 8 * cols - 8 * rows (what x and y leave of the 256 MiB
// Infinity Cache) load with the default cache policy and stay resident across
// launches; the rest non-temporal.  C4 shard (x 134 MB, 6.3 MB of entries per
// block), profiles/r06/wgs/wgs_nt_*.log: 0 / 6 / 9 / 12 / 15 / 18 / 20 / 28
// blocks resident 358.0 / 353.1 / 352.5 / 350.8 / 349.2 / 352.3 / 358 / 401 us;
// this budget gives 14 blocks (88 MB).
constexpr uint64_t kWgSplitMallBytes = 232ull << 20;
// Row blocks per k_wgather launch (option "wgather_chunk"): one per CU.  A
// matrix with more blocks than that (full C4: 2048 blocks of 8192 rows) runs
// in several launches, so every launch's workgroups are resident together
// and walk the x windows in step (one L2-resident window at a time); in one
// launch, later blocks start at window 0 while earlier ones are deep into x
// and the chip's gathers spread over many windows.  Full C4 on one GPU
// (profiles/r03/logs/sweep_c4_s7.log): one launch 6468 us, chunks of 1024
// 5287, 512 (two per CU) 4078, 256 (one per CU) 3620.
constexpr uint32_t kWgChunk = 256;
// Entry bytes of a vcache layout kept resident in the Infinity Cache across
// launches (capi.cpp resident_blocks): half of the 384 MiB of C3's entries
constexpr uint64_t kVcResidentBytes = 192ull << 20;
constexpr int kVcThreads = 1024;
constexpr int kVcSegMax = 256;        // npad + 1 <= kVcSegMax per unit
constexpr int kVcEpt = 2;             // entries per thread held in registers per panel
constexpr int kVcDepth = 4;           // panels of prefetch in flight (entries + x)
constexpr uint32_t kVcCont = 1u << 30;  // entry continues the previous entry's row run
constexpr uint32_t kVcMore = 1u << 31;  // next entry continues this entry's row run
// AUTO uses a vcache-family kernel only when no row has more than kVcRunMax
// entries inside one segment: a run is walked by one lane, one dependent load
// per entry (R-MAT s20 with hub rows: 23.6 ms in k_vcache split against
// 0.25 ms in csr_vector, round-2 sweep).
constexpr uint32_t kVcRunMax = 16;
// build_vcache_lanes / k_vquad: the entry's run continues in the same lane's
// next slot (position + CT), not in the next lane
constexpr uint32_t kVqLMore = 1u << 28;
// the k_vquad geometry: 16384 rows, 1984-column panels, 4 parts, 12 column
// bits (the code holds row_local << 12 and the flags in bits 28-31)
constexpr VcGeom kVcQuad{16384, 1984, 4, 12};
// ---- k_vflow (csrc/vflow.hip): four column parts of
// 16384-row blocks (x per CU a quarter of x, 64 x 4 = 256 units on C3); x in a
// ring of kVfSlots panels of 1280 columns handed from the loader waves to the
// compute waves by LDS flags instead of a workgroup barrier per step.  Compute
// wave w owns the block rows with vf_wave_of(row_local) == w -- every update of
// a y row comes from one wave, in step order, so waves may be at different
// steps.  LDS: 16384 * 8 + 3 * 1280 * 8 + 64 flag bytes.
constexpr VcGeom kVfGeom{16384, 1280, 4, 16, 4096};
constexpr int kVfLoaders = 2, kVfWaves = 14, kVfSlots = 3;
constexpr uint32_t kVfGroupMax = 128;  // entries of one (step, wave) group: two 64-lane slots
constexpr uint32_t vf_wave_of(uint32_t row_local) { return (row_local >> 5) % (uint32_t)kVfWaves; }
constexpr uint32_t kVqLanes = 13 * 64;
// k_vcache's split geometry: compute lanes (16 - 3 loader waves) * 64 (VcCfg<3>)
constexpr uint32_t kVcSplitCT = 13 * 64;
// ... and its ordered geometry's: (16 - 8 loader waves) * 64 (VcCfg<1>)
constexpr uint32_t kVcOrderedCT = 8 * 64;
// ... and its register-staged x loader waves (VcCfg<1>::WL; build_xmask's word per wave)
constexpr uint32_t kVcOrderedLoaders = 8;
// ... and its four-part geometry's: (16 - 2 loader waves) * 64 (VcCfg<4>)
constexpr uint32_t kVcSplit4CT = 14 * 64;  // k_vquad's compute lanes (13 of 16 waves): the layout's CT

// ---- wcsr: csr_vector over the column-windowed segment matrix
// Every row is cut at column windows of 2^kWcLog2Window columns (8 MiB of
// x); the pieces ("segments", one per (window, row) pair that has
// entries) form the rows of A', in window-major order.  csr_vector over A'
// walks x one window at a time; y[r] is the sum of r's segment partials in
// window order (k_wreduce).  One width for every matrix (a width that depends
// on the shard could cut a row differently in two partitions).  Round 4, C5
// 8-way cost partition, slowest shard / fastest (profiles/r04/logs
// bench_c5_cost.log, bench_c5_w*.log): 2^17 309.5 / 288.3 us, 2^18 297.2,
// 2^19 286.0, 2^20 283.2 / 271.3, 2^21 293.9, 2^22 319.2 -- fewer segments
// (shard 7: 11.8 M at 2^17, 6.6 M at 2^20) against gathers over more of x.
constexpr uint32_t kWcLog2Window = 20;
// AUTO considers wcsr from this many columns (x of 16 MiB: four XCD L2s)
// wcsr LDS form (k_wseg, opt-in HIPSPMV_WCSR_LDS=1): x windows of 2^14 f64
// (128 KiB of LDS), chunks of at most kWsChunkNnz entries of one window per
// 1024-thread workgroup
constexpr uint32_t kWsLog2Window = 14;
constexpr uint32_t kWsChunkNnz = 49152;
// wcsr hot-column form (round 6): per 2^kWcLog2Window window
// the K most frequent columns of the layout's entries (R-MAT: 16384 of 2^20
// columns carry ~60 % of a window's entries) are staged in LDS by each
// workgroup of the segment pass; their entries' colind become kWcHotFlag |
// slot, the rest gather from global memory as before.
constexpr uint32_t kWcHotFlag = 1u << 31;
constexpr uint32_t kWcHotMax = 16384;
constexpr uint32_t kWcMinCols = 1u << 21;

// ---- csr_vector geometry ---------------------------------------------------
constexpr int kCvGroupNnz = 256;  // max nnz of a multi-row group (4 per lane)
constexpr int kCvGroupRows = 64;  // max rows of a multi-row group (1 per lane)

// ---- k_sell geometry ---------------------------------------
// SELL-C-sigma: rows sorted by length (descending, stable) inside windows of
// kSellSigma rows, cut into slices of kSellRows rows, one wave per slice: lane
// l owns rows l, l+64, l+128, l+192 of the slice (four independent sequential
// sums per lane); entry k of sub-slice j, lane l at off + (4k + j)*64 + l.
// Rows longer than kSellHub entries are "hub" rows: one wave each, reading
// the CSR copy (ordered: one sequential chain; fast: lane partials + a fixed
// shuffle tree).
constexpr int kSellRows = 256;
constexpr uint32_t kSellSigma = 65536;
constexpr uint32_t kSellHub = 256;
constexpr uint32_t kSellNoRow = 0xFFFFFFFFu;
// FAST / u64: a hub row is cut into pieces of at most kSellPiece entries, one
// wave each; the wave that finishes a row's last piece (ticket) adds the
// piece partials in piece order (deterministic).  Piece record, 8 x u32:
// row, first entry (within the row), entries, piece index, pieces of the row,
// ticket index, 0, 0.
constexpr uint32_t kSellPiece = 4096;
// ORDERED f64: a hub row's chain holds kChainG consecutive entries per lane per
// stage of 64 * kChainG (csrc/sell.hip hub_row_exact; tools/sell_sim.cpp).
constexpr int kChainG = 8;
// ORDERED f64, k_sell_iso: hub rows of at least kSellIso entries get a
// 1024-thread workgroup each -- one chain wave alone on its SIMD, fed from
// LDS by 12 helper waves (csrc/sell.hip hub_row_isolated)
constexpr uint32_t kSellIso = 8192;
// products per chain lane per stage there: 45 * 64 = 2880, three per
// helper thread (all 15 other waves help; C5 shard 0 ORDERED 461 us, the
// longest row's chain at 4.6 cycles per add; G = 12 with 12 helper waves:
// 579-616 us)
constexpr int kIsoG = 45;
constexpr int kSellPieceWords = 8;

// Column part h of a geometry with `split` parts owns panels
// [vc_part_first(h), vc_part_first(h + 1)): floor cuts, so the parts differ by
// at most one panel and every part owns one as soon as npanels >= split (a
// ceil cut left the last of three parts empty for 4 panels, 12001-16000
// columns).  constexpr: the same function on the host (plan.cpp, vc_sim) and
// in the kernels.
constexpr uint32_t vc_part_first(uint32_t h, uint32_t npanels, uint32_t split) {
  return (uint32_t)((uint64_t)h * npanels / split);
}

// Launch geometry of a vcache-family kernel (k_vcache, k_wgather): true iff
// every work unit's rows and panels lie inside the matrix for a kernel
// compiled for geometry g -- the row-block bound, no surplus blocks (a block
// with r0 >= rows would compute rows - r0 in uint32 and write past y: the
// round-1 GPU fault), every column covered by the panels, every
// column part non-empty (npanels >= split), part_panels the largest part, and
// the unit's segment table inside LDS.  launch_vcache / launch_wgather return
// hipErrorInvalidValue without a launch when it is false; tools/vc_sim.cpp
// checks it on the CPU (incl. the incident geometry).
inline bool vcache_grid_ok(uint32_t rows, uint32_t cols, uint32_t rows_per_block, uint32_t nblocks,
                           uint32_t npanels, uint32_t part_panels, uint32_t npad, uint32_t panel, int split,
                           const VcGeom& g) {
  if (split != g.split || panel != (uint32_t)g.panel) return false;
  if (rows == 0 || cols == 0 || nblocks == 0 || rows_per_block == 0 || rows_per_block > (uint32_t)g.rows)
    return false;
  if ((uint64_t)nblocks * rows_per_block < rows) return false;         // every row in some block
  if ((uint64_t)(nblocks - 1) * rows_per_block >= rows) return false;  // no surplus block
  if (npanels == 0 || (uint64_t)npanels * g.panel < cols) return false;
  if (npanels < (uint32_t)split) return false;                         // every part owns a panel
  if (part_panels != (npanels + split - 1) / split) return false;      // the largest part
  return npad + 1 <= (uint32_t)g.segmax && npad >= part_panels;
}

// Host arrays the size of the matrix: resize() leaves new elements
// uninitialised (no single-threaded zero fill -- the builders write every
// element, from several threads, so the pages are first touched in parallel).
template <class T>
struct UninitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = UninitAlloc<U>;
  };
  UninitAlloc() = default;
  template <class U>
  UninitAlloc(const UninitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... args) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(args)...);
  }
};
template <class T>
using hvec = std::vector<T, UninitAlloc<T>>;

// Worker threads of the host-side builders: $HIPSPMV_THREADS, else
// $OMP_NUM_THREADS, else min(16, hardware threads) (plan.cpp).
unsigned plan_threads();

// A host array that owns its elements (hvec) or borrows the caller's: create
// from a CSR the caller holds reads it in place instead of copying it (the
// host CSR lives only for the duration of the create call).  Writes go
// through the owning storage; a borrowed array is read-only.
template <class T>
class HArr {
 public:
  HArr() = default;
  HArr(const HArr& o) { *this = o; }
  HArr& operator=(const HArr& o) {
    if (this != &o) {
      own_.assign(o.begin(), o.end());
      sync();
    }
    return *this;
  }
  HArr(HArr&& o) noexcept { *this = std::move(o); }
  HArr& operator=(HArr&& o) noexcept {
    const bool borrowed = o.p_ != o.own_.data();
    own_ = std::move(o.own_);
    p_ = borrowed ? o.p_ : own_.data();
    n_ = o.n_;
    o.own_.clear();
    o.p_ = nullptr;
    o.n_ = 0;
    return *this;
  }
  void borrow(const T* p, size_t n) {
    hvec<T>().swap(own_);
    p_ = const_cast<T*>(p);
    n_ = n;
  }
  void resize(size_t n) {
    own_.resize(n);
    sync();
  }
  void assign(size_t n, const T& v) {
    own_.assign(n, v);
    sync();
  }
  template <class It>
  void assign(It b, It e) {
    own_.assign(b, e);
    sync();
  }
  void clear() {
    own_.clear();
    sync();
  }
  void push_back(const T& v) {  // owning arrays only (tools that build a matrix row by row)
    own_.push_back(v);
    sync();
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  const T* data() const { return p_; }
  T* data() { return p_; }
  const T& operator[](size_t i) const { return p_[i]; }
  T& operator[](size_t i) { return p_[i]; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }
  T* begin() { return p_; }
  T* end() { return p_ + n_; }
  const T& front() const { return p_[0]; }
  const T& back() const { return p_[n_ - 1]; }
  bool operator==(const HArr& o) const { return n_ == o.n_ && std::equal(begin(), end(), o.begin()); }

 private:
  void sync() {
    p_ = own_.data();
    n_ = own_.size();
  }
  hvec<T> own_;
  T* p_ = nullptr;
  size_t n_ = 0;
};

struct HostCSR {
  uint32_t rows = 0, cols = 0, nnz = 0;
  HArr<uint32_t> rowptr, colind;
  HArr<uint64_t> vals;  // 8-byte words (f64 bits or u64)
};

struct VcacheLayout {
  VcGeom geom{};
  uint32_t rows_per_block = 0, nblocks = 0, npanels = 0;
  uint32_t part_panels = 0;  // panels of the largest column part (vc_part_first cuts: parts differ by <= 1)
  uint32_t npad = 0;         // seg entries per unit - 1 (= part_panels)
  std::vector<uint32_t> seg;    // (nblocks * split) units * (npad + 1) global entry offsets
  hvec<uint32_t> code;          // per entry: col_local | row_local << 16 | CONT | MORE
  hvec<uint64_t> vals;          // per entry
  uint32_t max_seg = 0;
  uint32_t max_run = 0;  // longest run of one row inside one segment
  uint64_t n_cont = 0;   // entries continuing a run (added after another entry of their row in one step)
  bool row_runs = false;  // place_segments_banked: every run inside one 16-lane DPP row of one wave
};

struct WinLayout {
  uint32_t log2w = 0, nseg = 0, max_seg = 0;
  std::vector<uint32_t> winseg;  // windows + 1: window w's segments are [winseg[w], winseg[w+1])
  HostCSR seg;                  // A': rows = segments (window-major, then row), cols = the matrix's
  hvec<uint32_t> rowseg;        // rows + 1: row r's segments are segidx[rowseg[r] .. rowseg[r+1])
  hvec<uint32_t> segidx;        // nseg: segment ids of each row, in window order
};

struct SellLayout {
  uint32_t nslices = 0, nhubs = 0, niso = 0;
  std::vector<uint64_t> off;    // nslices + 1: first entry of each slice
  std::vector<uint32_t> width;  // nslices: longest row of the slice
  hvec<uint32_t> row;           // nslices * kSellRows: row id (kSellNoRow past the window's rows)
  hvec<uint32_t> len;           // nslices * kSellRows: row length (0 for kSellNoRow)
  hvec<uint32_t> col;           // off[nslices] entries; padding: column 0
  hvec<uint64_t> vals;          // padding: 0 (never added: k < len selects)
  std::vector<uint32_t> hubs;   // hub rows, longest first (ORDERED: one wave each)
  std::vector<uint32_t> pieces; // FAST: kSellPieceWords per piece, pieces of a row contiguous
  uint32_t npieces = 0, ntickets = 0;
  uint64_t padding = 0;         // padded entries (off[nslices] - nnz of the slices)
};

// CSC (SparseMatrix layout) -> CSR, stable, masking bits 30-31 of the row ids.
// Returns a HIPSPMV_* status; fills `why` on validation failure.
int csc_to_csr(const uint32_t* colptr, const uint32_t* rowind, const void* vals, uint32_t rows, uint32_t cols,
               uint32_t nnz, HostCSR& out, std::string& why);
// CSR given by the caller: validated, then borrowed (out reads the caller's
// arrays, which must outlive it -- the create call).
int copy_csr(const uint32_t* rowptr, const uint32_t* colind, const void* vals, uint32_t rows, uint32_t cols,
             uint32_t nnz, HostCSR& out, std::string& why);

bool vcache_eligible(const HostCSR& a, const VcGeom& g);
// The block / panel / part geometry build_vcache will use, without the entries
// (rows_per_block, nblocks, npanels, part_panels, npad).
void vcache_geometry(uint32_t rows, uint32_t cols, const VcGeom& g, VcacheLayout& out);
uint32_t vcache_max_run(const HostCSR& a, uint32_t panel);
// by_line: each segment's row runs in x-line order (k_wgather; = sort_segments_by_line after)
void build_vcache(const HostCSR& a, const VcGeom& g, VcacheLayout& out, bool by_line = false);
// k_wgather's segment order: row runs by the x line of their first column (plan.cpp)
void sort_segments_by_line(VcacheLayout& L);
// k_vcache split: entries of each segment re-placed for LDS banks (plan.cpp;
// the same sums, bit-identical results)
void place_segments_banked(VcacheLayout& L, uint32_t CT);
struct VflowLayout {
  VcacheLayout L;              // blocks, panels, parts; entries regrouped by (unit, step, wave)
  hvec<uint32_t> wbeg, wend;   // [unit][wave][step < npad]: the group's entries [wbeg, wend)
  uint32_t max_group = 0;
};
// false: not eligible (a group past kVfGroupMax entries, or a run that cannot
// stay inside a 16-lane DPP row)
bool build_vflow(const HostCSR& a, VflowLayout& out);
// k_vquad's placement of the same entries for CT compute lanes (plan.cpp)
bool build_vcache_lanes(const HostCSR& a, const VcGeom& g, uint32_t CT, VcacheLayout& out);
// The ordered geometry's x-line mask (k_vcache SPLIT 1, register-staged loaders): per unit, panel
// and loader wave w (of WL), bit 8 j + k set when an entry of the unit's panel reads a column of x
// line w * 8 + j * 8 * WL + k (16 columns of 8 bytes per line).  out: units * npanels * WL words.
void build_xmask(const VcacheLayout& L, uint32_t WL, std::vector<uint64_t>& out);
void build_sell(const HostCSR& a, SellLayout& out);
// The column-windowed segment matrix of `a` (columns sorted within each row:
// vcache_eligible's condition).  Throws std::bad_alloc on host OOM.
// by_line: inside a window, segments ordered by the x line of their first
// column (then row), so a wave's gathers share lines; else by row
void build_windowed(const HostCSR& a, uint32_t log2w, WinLayout& out, uint32_t cap = UINT32_MAX,
                    bool by_line = false);
// The hot-column form of a global-x windowed layout: for each window w, its
// K most frequent columns ascending at hot[w * K ...] (padded with column 0),
// and every entry of such a column rewritten to kWcHotFlag | its slot.  The
// sums are unchanged (the same x values, read from LDS).  False (layout
// untouched) when a column id would collide with the flag.
bool mark_hot_columns(WinLayout& L, uint32_t K, std::vector<uint32_t>& hot);
// Segments build_windowed would make (one pass, no allocation).
uint64_t windowed_segments(const HostCSR& a, uint32_t log2w);
// Cost-balanced contiguous row partition (plan.cpp; hipspmv_partition_rows):
// bounds[parts + 1], interior bounds at multiples of HIPSPMV_SHARD_ALIGN.
void partition_rows_cost(const uint32_t* rowptr, const uint32_t* colind, uint32_t rows, uint32_t parts,
                         uint32_t* bounds);
// Row groups for csr_vector: group g covers rows [groups[g], groups[g+1]).
void build_row_groups(const HostCSR& a, std::vector<uint32_t>& groups);
void build_row_groups(const uint32_t* rowptr, uint32_t rows, std::vector<uint32_t>& groups);

// hipspmv_last_error() text for this thread (capi.cpp).
void set_last_error(const std::string& what);
// Releases device buffers, events (hipEvent_t) and streams (hipStream_t) of a
// destroyed object on the library's release thread, once the device has
// finished the work submitted before this call; returns at once (capi.cpp).
void defer_release(int device, std::vector<void*> ptrs, std::vector<void*> events, std::vector<void*> streams);

// csrc/prep.hip: the bodies of hipspmv_prep_stats / hipspmv_mark_row_starts.
int prep_stats(const uint32_t* colptr, const uint32_t* rowind, uint32_t rows, uint32_t cols, uint32_t nnz,
               int device, hipspmv_prep_stats_t* out);
int mark_row_starts(const uint32_t* rowind, uint32_t* rowind_out, uint32_t rows, uint32_t nnz, int reverse,
                    int shift, int device, uint64_t* kernel_ns);

}  // namespace hipspmv
