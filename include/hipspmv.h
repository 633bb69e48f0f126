/*
 * hipspmv.h -- C ABI of libhipspmv.so, the MI355X (gfx950) SpMV backend.
 *
 * This is the drop-in boundary behind the reference's plugin surface
 * (maltanar/spmv-vector-cache, software/): the HIPSpMV backend
 * (spmv-vector-cache_amd/host/HIPSpMV.cpp), registered in HWSpMVFactory, calls
 * it in place of the FPGA register drivers (software/SpMVAccelerator*Driver.hpp)
 * and the Chisel SpMVAccelerator* RTL they program.  Plain C types only: no HIP
 * or torch types appear in any signature (streams travel as void*).
 *
 * Each entry point names the reference interface it replaces.  All functions
 * return an int status (HIPSPMV_OK == 0) and never throw.
 *
 * Semantics follow SoftwareSpMV::exec (software/SoftwareSpMV.cpp:50-70):
 *   beta == 1 : y_out = y_in + A*x  (the reference's "y +=", accumulating into
 *               the caller's y, which main.cpp:220-222 zeroes beforehand)
 *   beta == 0 : y_out = A*x         (accumulator starts at +0.0, i.e. the
 *               reference's result on a zeroed y)
 * Rows without nonzeros keep y_in (beta 1) or get +0.0 (beta 0).
 *
 * Modes:
 *   HIPSPMV_MODE_ORDERED : every row is summed sequentially in ascending column
 *                          order, products rounded before each add (no FMA):
 *                          bit-identical to SoftwareSpMV for f64, and for u64.
 *   HIPSPMV_MODE_FAST    : f64 row sums may be reassociated (wave-level
 *                          segmented reduction); per row
 *                          |y - y_ref| <= 2*len*2^-53*sum|a_ij*x_j| (+ |y_in|
 *                          term for beta 1).  u64 stays bit-exact (mod 2^64).
 *   HIPSPMV_MODE_AUTO    : ORDERED (the default used for parity).
 */
#ifndef HIPSPMV_H_
#define HIPSPMV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIPSPMV_ABI_VERSION 1

/* status codes */
#define HIPSPMV_OK 0
#define HIPSPMV_ERR_INVALID_ARG 1    /* null pointer, bad enum, bad size */
#define HIPSPMV_ERR_INVALID_MATRIX 2 /* pointers not monotone, index out of range */
#define HIPSPMV_ERR_HIP 3            /* a HIP runtime call failed (see hipspmv_last_error) */
#define HIPSPMV_ERR_OOM 4            /* host or device allocation failed */
#define HIPSPMV_ERR_UNSUPPORTED 5    /* kernel/option not applicable to this matrix */
#define HIPSPMV_ERR_NO_DEVICE 6      /* requested device does not exist */
#define HIPSPMV_ERR_KEY 7            /* unknown stat / option key */

/* element types (SparseMatrix.h:6 SpMVData = double; u64 = StagedUIntOp
 * semiring of chisel/frontend/SemiringOp.scala:74-92) */
#define HIPSPMV_F64 0
#define HIPSPMV_U64 1

#define HIPSPMV_MODE_AUTO 0
#define HIPSPMV_MODE_ORDERED 1
#define HIPSPMV_MODE_FAST 2

/* kernel selection (option "kernel") */
#define HIPSPMV_KERNEL_AUTO 0
#define HIPSPMV_KERNEL_VCACHE 1     /* x panels + y block staged in LDS; ordered */
#define HIPSPMV_KERNEL_CSR_LANE 2   /* one lane per row over CSR; ordered */
#define HIPSPMV_KERNEL_CSR_VECTOR 3 /* wave segmented DPP reduction over CSR; fast */
#define HIPSPMV_KERNEL_VCACHE_SPLIT 4 /* vcache over three column parts, fixed-order
                                         combine p0 + p1 + p2; fast, deterministic */
#define HIPSPMV_KERNEL_VCACHE_SPLIT4 5 /* four column parts, p0+p1+p2+p3; fast,
                                          deterministic; never chosen by AUTO,
                                          its layout is built on first selection
                                          by name (option "kernel", or the stat
                                          "vcache_split4_eligible") */
#define HIPSPMV_KERNEL_WGATHER 6 /* y block in LDS, x gathered from global in
                                    2^16-column windows (wide x: C4);
                                    ordered; chosen by AUTO for wide x */
#define HIPSPMV_KERNEL_WCSR 8 /* csr_vector over the rows cut at 2^20-column
                                 windows (window-major), then each row's window
                                 partials summed in a fixed order; fast,
                                 deterministic; wide, skewed x (C5 shards) */
#define HIPSPMV_KERNEL_VCACHE_FLOW 9 /* "vcache_flow": the vector cache over four column
                                  parts of 16384-row blocks, x in a 3-slot LDS ring
                                  handed over by LDS flags (no workgroup barrier per
                                  step), each compute wave owning its y rows;
                                  fast, deterministic; layout built on first
                                  selection (stat "vflow_eligible") */
#define HIPSPMV_KERNEL_SELL 7 /* SELL-C-sigma: one lane per row over slices of
                                 256 length-sorted rows, coalesced entries; rows
                                 over 256 entries one wave each (ORDERED: rows of
                                 8192+ entries as isolated chains, a 1024-thread
                                 workgroup each); ordered in ORDERED mode (FAST:
                                 long rows cut into pieces); any matrix */
#define HIPSPMV_KERNEL_WGATHER_SPLIT 10 /* "wgather_split": k_wgather over two column
                                  halves of 16384-row blocks (part 0 on XCDs 0-3,
                                  part 1 on XCDs 4-7; option "wgather_map" 1
                                  alternates them), y = p0 + p1; fast,
                                  deterministic; chosen by AUTO (FAST) for wide x
                                  with at most 2^21 rows (a C4 shard) */

typedef struct hipspmv_handle hipspmv_t;

/* Replaces HardwareSpMV construction + setupRegs()
 * (software/HardwareSpMV.cpp:8-25, HardwareSpMVNewCache.cpp:31-44): takes the
 * SparseMatrix CSC arrays (SparseMatrix.h:36-58: indPtrs = colptr[cols+1],
 * inds = row ids[nnz], nzData = 8-byte values[nnz]) and builds the device
 * copy.  Bits 30-31 of the row ids (cold-miss-skip marks,
 * SparseMatrix.cpp:52-90) are masked off; the caller's arrays are never
 * modified and may be freed after the call.  device is a HIP ordinal. */
int hipspmv_create(const uint32_t *colptr, const uint32_t *rowind, const void *vals, uint32_t rows,
                   uint32_t cols, uint32_t nnz, int dtype, int device, hipspmv_t **out);

/* Same, from CSR arrays (rowptr[rows+1], colind[nnz], vals[nnz]); colind need
 * not be sorted within a row for FAST mode, and is summed in the given order
 * for ORDERED mode.  Used for row-partitioned shards. */
int hipspmv_create_csr(const uint32_t *rowptr, const uint32_t *colind, const void *vals, uint32_t rows,
                       uint32_t cols, uint32_t nnz, int dtype, int device, hipspmv_t **out);

/* Options: "kernel" (HIPSPMV_KERNEL_*), "mode" (default mode for exec with
 * HIPSPMV_MODE_AUTO), "timing" (1 = record per-exec kernel events),
 * "vcache_dma" (-1 default; 1 = vcache kernels stage x by LDS-DMA; the
 * VCACHE_SPLIT geometry always does), "vcache_xlane" (-1 default: 5 (else 3) for
 * VCACHE_SPLIT, 0 otherwise; 1 = vcache run continuations across lanes
 * instead of reloads; 2 = that plus step loops padded to the unroll and
 * register rings loaded by inline asm with explicit vmcnt waits; 3 =
 * cross-lane and padded loops with the compiler's own waits -- 2 and 3 keep
 * the DE-deep entry prefetch in flight across the loop header; 5 = 3 with the
 * first continuation step by DPP, for VCACHE_SPLIT layouts whose runs stay in
 * 16-lane rows -- the default there; 6 = VCACHE (ordered) on such a layout:
 * the first continuation entry from the next lane by DPP, entry loads past a
 * step masked -- the same bits, measured no faster), "vcache_map"
 * (1 = VCACHE_SPLIT4 places column part h on XCDs 2h and 2h+1, so each XCD's
 * L2 serves a quarter of x; experimental), "profile" (1 = VCACHE and
 * VCACHE_SPLIT launches run in their default configuration with in-kernel
 * stamps, and the NewCache state statistics below are measured; results are
 * bit-identical to the unprofiled kernel), "vcache_nt" (row blocks b >=
 * vcache_nt of VCACHE / VCACHE_SPLIT load their entries non-temporally, the
 * blocks before them stay in the Infinity Cache across launches; -1 default:
 * about 192 MiB of entries resident -- C3: half the blocks of either; WGATHER:
 * 0 or -1 non-temporal, > 0 the default policy; WGATHER_SPLIT: the first
 * non-temporal row block, -1 the leading blocks that fit 232 MiB less x and y),
 * "wgather_chunk" (row blocks per WGATHER launch, 256 default; WGATHER_SPLIT
 * halves it per launch: two units per block), "wgather_map" (WGATHER_SPLIT:
 * 0 default, column half 0 on XCDs 0-3 and half 1 on 4-7; 1 alternating; the
 * same bits), "wcsr_xcd" (1 = WCSR's segment pass placed by XCD eighths of its
 * window order; the same bits; 0 default), "sell_nt" (SELL slices s >=
 * sell_nt likewise; -1 default: the second half).  The cache policy never
 * changes a result bit.  "vcache_xmask" (1 default: VCACHE's x loaders skip
 * the 128-byte x lines no entry of a unit's panel uses; 0 = load every line;
 * the same bits).  "wcsr_reduce" (0 default: WCSR's reduce runs over the rows
 * that have segments and fills the others; 1 = over every row; both
 * deterministic, their FAST bits may differ).  "vquad_variant" (VCACHE_SPLIT4 configuration,
 * csrc/vquad.hip: 0 default; 1-5, 17-19 other x / entry ring depths; 20 every
 * column-part owner gives up waiting, so the publish-and-count combine runs --
 * exact, counted by the stat "handoff_fallbacks"; 21 XCD placement; 22 / 23
 * with / without it, the entries of row blocks below "vcache_nt" in the
 * Infinity Cache; 24-26 y updated by LDS atomics; 6-16 are timing ablations
 * whose y is wrong: HIPSPMV_EXPERIMENTAL=1 only).  Experimental (HIPSPMV_EXPERIMENTAL=1): "sell_chain"
 * (ORDERED hub chains: 1 = no isolated chains, 2 / 3 = isolated stages of 12 /
 * 30 products per lane instead of 45; the same bits), "sell_only" (timing
 * probe, y incomplete: 1 hub rows only, 2 slices only, 3 the longest row). */
int hipspmv_set_option(hipspmv_t *h, const char *key, int64_t value);

/* Replaces HardwareSpMV::exec()'s reset -> init -> regular -> write sequence
 * (HardwareSpMVNewCache.cpp:78-101): copies x (cols elements) to the device,
 * runs the kernel, copies y (rows elements) back, synchronously.  y is read
 * first when beta == 1. */
int hipspmv_exec(hipspmv_t *h, const void *x, void *y, int beta, int mode);

/* Device-resident variant: d_x, d_y_in and d_y_out are device pointers on the
 * handle's device; enqueued on `stream` (a hipStream_t; NULL is HIP's default
 * stream, as in every HIP API) and returns without synchronising.  d_y_in may
 * equal d_y_out and is ignored for beta == 0.  Concurrency: a handle is used
 * from one host thread at a time.  Launches of one handle on different streams
 * may be in flight together: the kernels that combine partial sums through
 * scratch memory (VCACHE_SPLIT, VCACHE_SPLIT4, WCSR, SELL in FAST / u64 with
 * hub pieces) get one scratch set per stream (told apart by the stream value;
 * hipspmv_exec's internal stream has its own), so launches on different streams
 * share nothing and the handle records or waits on nothing between launches --
 * a stream may be destroyed right after its last launch.  Up to four streams
 * keep their sets; a fifth takes over the least recently used set after a
 * device synchronisation (stat "scratch_evictions").  Inside a stream capture
 * nothing is allocated or synchronised: the captured launch uses the capturing
 * stream's set if a launch on that stream made one, else the first set, and the
 * caller orders a graph's replays against the handle's other launches. */
int hipspmv_exec_device(hipspmv_t *h, const void *d_x, const void *d_y_in, void *d_y_out, int beta, int mode,
                        void *stream);

/* Replaces HardwareSpMV::statInt/statKeys (HardwareSpMV.cpp:41-61,
 * HardwareSpMVNewCache.cpp:130-204).  Keys: "rows" "cols" "nz" "dtype"
 * "device" "kernel" (last kernel run) "setup_ns" "create_ns" "layout_ns"
 * "setup_csr_ns" "setup_upload_ns" "setup_scan_ns" "setup_layouts_ns"
 * (create's phases) "kernel_ns" (last timed
 * exec) "h2d_ns" "d2h_ns" "alg_bytes" (beta 0) "alg_bytes_beta1" "flops"
 * "device_bytes" "vcache_blocks" "vcache_panels" "vcache_rows_per_block"
 * "vcache_max_segment" "vcache_eligible" "vcache_split_eligible"
 * "vcache_split_units" "vcache_split_rows_per_block" "vcache_x_bytes"
 * "vcache_split_x_bytes" (x bytes one launch streams into LDS)
 * "vcache_split4_eligible" "vcache_split4_x_bytes" "wgather_eligible"
 * "wgather_windows" "wgather_split_eligible" "wgather_split_rows_per_block"
 * "wgather_split_units" "row_groups" "sell_slices" "sell_hubs" "sell_hub_pieces"
 * "sell_padding" "sell_iso_hubs" (SELL layout, 0 until the sell kernel is
 * selected) "wcsr_segments" "wcsr_max_segment" "wcsr_window_log2"
 * "wcsr_chunks" (wcsr layout)
 * "resident_entry_bytes" (entry bytes the last launch loaded with the default
 * cache policy, which may stay in the Infinity Cache until the next launch;
 * the rest load non-temporally: options vcache_nt / sell_nt)
 * "scratch_streams" "scratch_evictions" (per-stream combine scratch sets, see
 * hipspmv_exec_device)
 * "max_row_len" "empty_rows" "execs" "handoff_fallbacks" (VCACHE_SPLIT4
 * combine owners that gave up waiting, since create); the reference accelerator's cache
 * statistics for the last launch: "total_cycles" "active_cycles" "read_misses"
 * "hazard_stalls" "ocm_depth" "issue_window" "capacity_stalls" "cms"; measured
 * by the last launch run with option "profile" (means over its workgroups, in
 * shader cycles; 0 before one): "state_fill" "state_active" "state_flush"
 * "state_done" "state_read_miss1" "state_read_miss2" "state_read_miss3"
 * "state_cold_miss" (the cache FSM states of NoWMVectorCache.scala:162)
 * "no_valid_but_ready" "no_ready_but_valid" (StreamMonitor stalls) "profiled"
 * "profile_units" "profile_span_cycles". */
int hipspmv_stat(hipspmv_t *h, const char *key, uint64_t *out);

/* Hardware counters behind the cache statistics (the reference reads its
 * counters from the accelerator after a run, HardwareSpMVNewCache.cpp:161-173).
 * hipspmv_pmc_counter: mean per dispatch of `counter` over the dispatches whose
 * kernel name contains `kernel` (NULL: any hipspmv kernel; the instantiation
 * with the most dispatches) in a rocprofv3 --pmc counter_collection.csv, or
 * the per_dispatch value of a tools/pmc_summary.py summary; no device needed.
 * hipspmv_attach_pmc: such a CSV (collected for this handle's kernel; NULL or
 * "" detaches) backs the stat keys "read_misses" (TCC_MISS), "hazard_stalls"
 * (SQ_LDS_BANK_CONFLICT) and "capacity_stalls" (TCP_PENDING_STALL_CYCLES) of
 * the last kernel when it holds them; "read_misses_model" and
 * "hazard_stalls_model" keep the layout values; "pmc_attached". */
int hipspmv_pmc_counter(const char *csv_path, const char *kernel, const char *counter, double *mean,
                        uint64_t *dispatches);
int hipspmv_attach_pmc(hipspmv_t *h, const char *csv_path);

/* Name of the kernel that HIPSPMV_MODE `mode` would run (static string). */
const char *hipspmv_kernel_name(hipspmv_t *h, int mode);

/* Replaces the HardwareSpMV destructor (software/HardwareSpMV.cpp:27).
 * Returns at once: the handle's device memory, events and stream are released
 * by the library's release thread once the device has finished the work
 * submitted before this call (launches of the handle on any stream, destroyed
 * streams included), so destroying a handle never makes the calling thread
 * wait for the device (hipFree would: an implicit device synchronisation).
 * The handle pointer is invalid on return. */
int hipspmv_destroy(hipspmv_t *h);

/* Blocks until every release queued by hipspmv_destroy / hipspmv_multi_destroy
 * so far has completed (the memory is back with the device allocator). */
int hipspmv_release_wait(void);

/* Matrix preprocessing statistics on the GPU.  Replaces
 * SoftwareSpMV::measurePreprocessingTimes (software/SoftwareSpMV.cpp:72-95)
 * and the SparseMatrix scans it times: maxColSpan (SparseMatrix.cpp:110-119),
 * maxAlive (SparseMatrix.cpp:92-108) and markRowStarts(false, 31)
 * (SparseMatrix.cpp:52-90, timed only).  Row ids are read with bits 30-31
 * masked, so the values are the reference's on an unmarked matrix (as
 * measurePreprocessingTimes runs them) even if A carries CMS marks.  Input is
 * the SparseMatrix CSC (colptr[cols+1], rowind[nnz]); times are GPU kernel
 * time in ns with the data resident (h2d_ns is the upload). */
typedef struct {
  uint32_t max_alive;
  uint32_t max_col_span;
  uint64_t max_alive_ns;
  uint64_t max_col_span_ns;
  uint64_t cms_ns;
  uint64_t h2d_ns;
} hipspmv_prep_stats_t;

int hipspmv_prep_stats(const uint32_t *colptr, const uint32_t *rowind, uint32_t rows, uint32_t cols, uint32_t nnz,
                       int device, hipspmv_prep_stats_t *out);

/* SparseMatrix::markRowStarts(reverse, shift) (SparseMatrix.cpp:52-90) on the
 * GPU: rowind_out[e] = rowind[e] | 1 << shift for the first (reverse: last)
 * entry of every row in storage order, other entries copied.  Rows are
 * compared with bits 30-31 masked; rowind_out may equal rowind.  kernel_ns
 * (may be NULL) receives the GPU time without the transfers. */
int hipspmv_mark_row_starts(const uint32_t *rowind, uint32_t *rowind_out, uint32_t rows, uint32_t nnz, int reverse,
                            int shift, int device, uint64_t *kernel_ns);

/* Row partitions: a block of rows handed to its own handle (a shard) gives
 * rows bit-identical to the unpartitioned matrix in every mode and kernel
 * when the block starts at a multiple of HIPSPMV_SHARD_ALIGN rows and runs
 * the same kernel (the FAST csr_vector kernel groups rows within aligned
 * 64-row windows; every other kernel is position-independent; ORDERED is
 * kernel-independent, FAST AUTO may choose by shard shape).  One exception:
 * WCSR in FAST f64 -- its segment pass groups the window-major segments of
 * all the shard's rows, so a row's partials depend on which other rows share
 * its windows; a shard's rows stay within the FAST bound but may differ in
 * the last bits from the unpartitioned run (u64 is exact either way; the
 * window width is the same for every matrix).  hipspmv_multi_create and the
 * host partition helpers cut at such rows. */
#define HIPSPMV_SHARD_ALIGN 64

/* Row partition used by hipspmv_multi_create (and bench.py's C5 shards):
 * `parts` contiguous blocks of about equal cost, a row costing its entries +
 * its segments at the wcsr kernel's 2^20-column windows (runs of more than 256
 * entries in a window cut into pieces) + 1, interior bounds snapped to the
 * nearer multiple of HIPSPMV_SHARD_ALIGN.  CSR input (rowptr[rows + 1],
 * colind[nnz]); writes bounds[parts + 1] (bounds[0] = 0, bounds[parts] =
 * rows).  Host only, no device.  Replaces the nnz-balanced partitionRows of
 * ref:software/main.cpp-style drivers for skewed matrices. */
int hipspmv_partition_rows(const uint32_t *rowptr, const uint32_t *colind, uint32_t rows, uint32_t cols,
                           uint32_t parts, uint32_t *bounds);

/* ---- several devices of one process ---------------------------------------
 * One matrix row-partitioned over ndev devices (rows cut into contiguous,
 * cost-balanced blocks by hipspmv_partition_rows; block i
 * on devices[i]): the single-host-thread
 * multi-GPU form of SURVEY.md §8(b)/(e), for HIPSpMV (register num_devices)
 * and C callers.  exec copies x to devices[0], broadcasts it device to device
 * (RCCL ncclBroadcast over xGMI when the ids are distinct, peer copies when an
 * id repeats), runs every block on its device and copies each block's y into
 * its rows of y.  No cross-device reduction: every row equals the
 * single-device result for the same mode and kernel.  Stat keys:
 * "num_devices" "rccl" "rows" "cols" "nz" "setup_ns" "h2d_ns" "bcast_ns"
 * "kernel_ns" (slowest block) "d2h_ns" "execs" "kernel" (block 0's last) "alg_bytes" (x counted once per
 * device) and "shard<i>_{rows,row0,nz,device,kernel_ns}". */
typedef struct hipspmv_multi hipspmv_multi_t;

int hipspmv_multi_create(const uint32_t *colptr, const uint32_t *rowind, const void *vals, uint32_t rows,
                         uint32_t cols, uint32_t nnz, int dtype, const int *devices, int ndev,
                         hipspmv_multi_t **out);
/* The same from a CSR (rowptr[rows + 1], colind[nnz] ascending within each
 * row, vals[nnz]); the arrays are read during the call only. */
int hipspmv_multi_create_csr(const uint32_t *rowptr, const uint32_t *colind, const void *vals, uint32_t rows,
                             uint32_t cols, uint32_t nnz, int dtype, const int *devices, int ndev,
                             hipspmv_multi_t **out);
/* Block i's own handle (NULL for a block without rows), owned by m: its
 * hipspmv_exec_device / hipspmv_stat run that block alone (per-block timing). */
int hipspmv_multi_shard(hipspmv_multi_t *m, int i, hipspmv_t **out);
int hipspmv_multi_set_option(hipspmv_multi_t *m, const char *key, int64_t value);
int hipspmv_multi_exec(hipspmv_multi_t *m, const void *x, void *y, int beta, int mode);
int hipspmv_multi_stat(hipspmv_multi_t *m, const char *key, uint64_t *out);
int hipspmv_multi_destroy(hipspmv_multi_t *m);

/* The measured HBM ceiling (not on the SpMV path; bench.py's second
 * denominator): a streaming copy (read + write counted) and a
 * streaming read of `bytes`-sized buffers on `device`, 16-byte non-temporal
 * accesses, `reps` timed launches each after two untimed ones.  Either output
 * may be NULL (that stream is then not run). */
int hipspmv_stream_bandwidth(int device, uint64_t bytes, int reps, double *copy_gbs, double *read_gbs);

const char *hipspmv_strerror(int status);
/* Text of the last HIP error seen by this thread (static per-thread buffer). */
const char *hipspmv_last_error(void);
int hipspmv_abi_version(void);
/* Build variant: HIPSPMV_BUILD_EXPERIMENTAL when the library carries the
 * kernel forms AUTO never picks (VCACHE_SPLIT4 / k_vquad, the vcache
 * continuation forms 1, 2, 4 and the ordered ones, "vcache_map", the ordered
 * LDS-DMA loader, "vquad_variant"): make EXPERIMENTAL=1 builds them into
 * lib/exp/libhipspmv.so.  The product library answers HIPSPMV_ERR_UNSUPPORTED
 * to the options and kernel that select them. */
#define HIPSPMV_BUILD_EXPERIMENTAL 1
int hipspmv_build_flags(void);
int hipspmv_device_count(int *count);

#ifdef __cplusplus
}
#endif
#endif
