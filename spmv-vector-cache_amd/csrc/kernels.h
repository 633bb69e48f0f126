// Kernel launch interface used by capi.cpp (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hipspmv {

struct VcacheArgs {
  const uint32_t* seg;
  const uint32_t* code;
  const void* vals;
  const void* x;
  const void* y_in;
  void* y_out;
  void* partial;       // split == 2: [2][rows] scratch for the column-part partials
  uint32_t* tickets;   // split == 2: [nblocks] arrival counters, zero between launches
  uint32_t rows, cols, rows_per_block, nblocks, npanels, part_panels, npad, last;
  int split, beta;
  int dma = 0;        // x panels by LDS-DMA (experimental loader, option "vcache_dma")
  uint32_t panel = 0; // the layout's panel width: checked against the kernel's
  int xlane = 0;      // cross-lane run continuation (experimental, option "vcache_xlane")
  uint32_t max_seg = 0;  // longest segment of the layout (xlane needs it in the register window)
  int map = 0;           // split 4: XCD-aware unit placement (experimental, option "vcache_map")
  uint32_t chunk = 0;    // k_wgather: row blocks per launch (0: one launch)
  uint32_t nt_from = ~0u;  // k_vcache: row blocks b >= nt_from load their entries non-temporally
  uint32_t* status = nullptr;  // k_vquad: bit 0 set when a combine hand-off wait timed out
  int variant = 0;             // k_vquad: configuration (loader waves, x / entry ring depths)
  bool row_runs = false;       // every run of the layout inside one 16-lane row (place_segments_banked):
                               // the split kernel's first continuation step by DPP (xlane 5)
  const uint64_t* xmask = nullptr;  // ordered geometry: the x lines each unit's panels use (build_xmask)
};

struct CsrArgs {
  const uint32_t* rowptr;
  const uint32_t* colind;
  const void* vals;
  const void* x;
  const void* y_in;
  void* y_out;
  const uint32_t* groups;
  uint32_t rows, ngroups;
  int beta;
};

struct WcsrArgs {  // csr_vector over the column-windowed segment matrix, then k_wreduce
  const uint32_t* seg_rowptr;
  const uint32_t* seg_colind;
  const void* seg_vals;
  const uint32_t* groups;  // csr_vector row groups of the segment matrix
  uint32_t ngroups;
  const uint32_t* rowseg;         // [rows + 1]: row r's segments are segidx[rowseg[r] .. rowseg[r+1])
  const uint32_t* segidx;         // [nseg]: each row's segment ids, in window order
  const uint32_t* reduce_groups;  // csr_vector row groups of the (rowseg, segidx) reduce
  uint32_t rgroups;
  void* ypart;                    // [nseg] segment partials, in segment order
  const void* x;
  const void* y_in;
  void* y_out;
  uint32_t rows;
  int beta;
  const uint32_t* chunks = nullptr;  // LDS form (k_wseg): (window, first group, end group) per workgroup
  uint32_t res_groups = 0;  // segment-pass groups g < res_groups load entries with the default policy
                            // (Infinity-Cache resident across launches; k_wpass), the rest non-temporal
  uint32_t nchunks = 0;
  uint32_t cols = 0;
  // the compact reduce (k_wreduce_c, used when rrow is set): groups over the rows that have segments
  // only -- rrow[i] is the i-th such row, rsegc[i] = rowseg[rrow[i]] (nrows_ne + 1 entries) -- and
  // the rows without any (bit r of nebits clear) written by the same launch's fill blocks
  const uint32_t* rrow = nullptr;
  const uint32_t* rsegc = nullptr;
  const uint32_t* nebits = nullptr;
  const uint32_t* cgroups = nullptr;
  uint32_t ncgroups = 0;
  int fill_early = 0;  // the rows without segments written by the segment pass's launch (k_wpass_fill)
  int xcd = 0;         // option wcsr_xcd: segment-pass blocks placed by XCD eighths of the window order
  // hot-column form (k_wpass_hot, needs chunks): [window][hotk] columns each workgroup stages in LDS;
  // entries with colind & kWcHotFlag read slot colind & ~kWcHotFlag of it
  const uint32_t* hot = nullptr;
  uint32_t hotk = 0;
};

struct SellArgs {
  const uint64_t* off;    // [nslices + 1]
  const uint32_t* width;  // [nslices]
  const uint32_t* row;    // [nslices * 256]
  const uint32_t* len;    // [nslices * 256]
  const uint32_t* col;    // padded entries
  const void* vals;
  const uint32_t* hubs;   // [nhubs] rows read from the CSR copy
  const uint32_t* rowptr;
  const uint32_t* colind;
  const void* csr_vals;
  const void* x;
  const void* y_in;
  void* y_out;
  uint32_t nslices, nhubs;
  int beta;
  int exact;  // 1: hub rows summed in one sequential chain (ORDERED f64)
  const uint32_t* pieces = nullptr;  // exact == 0: hub-row pieces (kSellPieceWords each)
  uint32_t npieces = 0;
  void* partial = nullptr;      // [npieces] piece partials
  uint32_t* tickets = nullptr;  // per split row, zero between launches
  uint32_t nt_from = 0;         // slices s >= nt_from load their entries non-temporally
  uint32_t niso = 0;            // hubs[0, niso): isolated chains (k_sell_iso)
  uint32_t chain_g = 0;         // exact: 0 product; 1 no isolated chains; 2 / 3 isolated stages of G = 12 / 30 (experimental)
};

struct VflowArgs {  // k_vflow (csrc/vflow.hip) over a build_vflow layout
  const uint32_t* wbeg;  // [unit][wave][npad]
  const uint32_t* wend;
  const uint32_t* code;
  const void* vals;
  const void* x;
  const void* y_in;
  void* y_out;
  void* partial;       // [4][nblocks][16384] column-part partials
  uint32_t* tickets;   // [4 * nblocks] combine share counters, zero between launches
  uint32_t* status;    // bit 1: a flag wait gave up (results wrong; never a hang)
  uint32_t rows, cols, rows_per_block, nblocks, npanels, part_panels, npad;
  int beta;
  uint32_t nt_from = ~0u;  // row blocks b >= nt_from load their entries non-temporally
  int map = 0;             // 1: XCDs 2h, 2h + 1 take column part h (vc_map.h MAP 1)
  int de = 4;              // steps of entries in flight per compute wave (2, 3, 4, 8)
  uint32_t* prof = nullptr;  // diagnostic stamps (option "vflow_prof"): 4 u32 per (unit, wave)
};
hipError_t launch_vflow(int dtype, const VflowArgs& a, hipStream_t s);

hipError_t launch_vcache(int dtype, const VcacheArgs& a, hipStream_t s);
// The same kernel in its default configuration (ordered: register-staged
// loaders; split 3: LDS-DMA loaders, cross-lane runs when the layout fits)
// with the profile stamps on (k_vcache AB bit 128): 8 u32 per workgroup at
// a.tickets + 4 * nblocks (split 3) or at a.partial (split 1).  Results are
// the default kernel's bits.  Split 4: hipErrorInvalidValue.
hipError_t launch_vcache_profiled(int dtype, const VcacheArgs& a, hipStream_t s);
constexpr int kVcProfWords = 8;
// k_vquad (csrc/vquad.hip): the four-part vector cache over the kVcSplit4
// layout, x panels DX deep in registers; needs a.status and max_seg within
// vquad_max_window(a.variant).
hipError_t launch_vquad(int dtype, const VcacheArgs& a, hipStream_t s);
uint32_t vquad_max_window(int variant);
hipError_t launch_sell(int dtype, const SellArgs& a, hipStream_t s);
hipError_t launch_wcsr(int dtype, const WcsrArgs& a, hipStream_t s);
// k_wgather over a kWgWindow layout (a.split 1, ORDERED), or over a kWgSplit
// layout (a.split 2, FAST: a.partial / a.tickets as k_vcache's split geometry)
hipError_t launch_wgather(int dtype, const VcacheArgs& a, hipStream_t s);
hipError_t launch_csr_lane(int dtype, const CsrArgs& a, hipStream_t s);
hipError_t launch_csr_vector(int dtype, const CsrArgs& a, hipStream_t s);

}  // namespace hipspmv
