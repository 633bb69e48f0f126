// libhipspmv.so: the C ABI of include/hipspmv.h.
//
// A handle owns the device copy of one matrix (CSR plus, when eligible, the
// vcache segment layout), the HIP stream it runs on by default, the staging
// buffers of the host-pointer exec path and its statistics.  Nothing here
// throws across the ABI: every entry point catches and returns a status.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <deque>
#include <fstream>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include "hipspmv.h"
#include "hipspmv_internal.h"
#include "kernels.h"

using namespace hipspmv;

namespace {

thread_local std::string g_last_error;

struct DeviceGuard {  // restore the caller's current device on scope exit
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? HIPSPMV_ERR_OOM : HIPSPMV_ERR_HIP;
}

#define HIP_TRY(call)                                        \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess) return hip_fail(e_, #call);        \
  } while (0)

template <typename T>
int dev_upload(T** dst, const T* src, size_t n, uint64_t& bytes) {
  *dst = nullptr;
  const size_t sz = sizeof(T) * (n ? n : 1);
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(dst), sz));
  bytes += sz;
  if (n) HIP_TRY(hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice));
  return HIPSPMV_OK;
}

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Deferred release: hipFree waits for the whole device
// (an implicit hipDeviceSynchronize), so a destroy on the caller's thread
// stalled every launch that thread had queued behind it -- a garbage-collected
// handle inside a timed loop reads as one 1.6 ms launch.  A
// destroyed handle's buffers, events and stream go to this thread instead: it
// waits for the device there (every launch submitted before the destroy,
// on any stream, live or destroyed since, has then finished) and frees them.
// The caller's thread never waits.  Drained at process exit (the object is
// constructed after the HIP runtime, so it is destroyed before it).
class Reclaimer {
 public:
  struct Item {
    int device = 0;
    std::vector<void*> ptrs;
    std::vector<hipEvent_t> events;
    std::vector<hipStream_t> streams;
  };
  static Reclaimer& get() {
    static Reclaimer r;
    return r;
  }
  void push(Item it) {
    std::unique_lock<std::mutex> lk(m_);
    if (!th_.joinable()) th_ = std::thread([this] { run(); });
    q_.push_back(std::move(it));
    ++queued_;
    cv_.notify_all();
  }
  // until everything pushed so far is released
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    const uint64_t target = queued_;
    done_cv_.wait(lk, [&] { return released_ >= target; });
  }
  ~Reclaimer() {
    {
      std::unique_lock<std::mutex> lk(m_);
      stop_ = true;
      cv_.notify_all();
    }
    if (th_.joinable()) th_.join();
  }

 private:
  void run() {
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop_ and drained
        it = std::move(q_.front());
        q_.pop_front();
      }
      (void)hipSetDevice(it.device);
      (void)hipDeviceSynchronize();  // this thread only
      for (void* p : it.ptrs)
        if (p) (void)hipFree(p);
      for (hipEvent_t e : it.events)
        if (e) (void)hipEventDestroy(e);
      for (hipStream_t s : it.streams)
        if (s) (void)hipStreamDestroy(s);
      std::unique_lock<std::mutex> lk(m_);
      ++released_;
      done_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::deque<Item> q_;
  std::thread th_;
  uint64_t queued_ = 0, released_ = 0;
  bool stop_ = false;
};

}  // namespace

void hipspmv::set_last_error(const std::string& what) { g_last_error = what; }

#ifdef HIPSPMV_EXPERIMENTAL_KERNELS
static constexpr bool kExperimental = true;
#else
static constexpr bool kExperimental = false;
#endif

void hipspmv::defer_release(int device, std::vector<void*> ptrs, std::vector<void*> events,
                            std::vector<void*> streams) {
  Reclaimer::Item it;
  it.device = device;
  it.ptrs = std::move(ptrs);
  for (void* e : events) it.events.push_back(static_cast<hipEvent_t>(e));
  for (void* s : streams) it.streams.push_back(static_cast<hipStream_t>(s));
  Reclaimer::get().push(std::move(it));
}

struct hipspmv_handle {
  int device = 0, dtype = HIPSPMV_F64;
  uint32_t rows = 0, cols = 0, nnz = 0;
  hipStream_t stream = nullptr;
  uint32_t *d_rowptr = nullptr, *d_colind = nullptr, *d_groups = nullptr;
  uint64_t* d_vals = nullptr;
  uint32_t ngroups = 0;
  struct Vc {  // one vcache layout on the device (ordered or split geometry)
    bool ok = false;
    uint32_t *d_seg = nullptr, *d_code = nullptr, *d_tickets = nullptr;
    uint64_t *d_vals = nullptr, *d_partial = nullptr;
    uint64_t* d_xmask = nullptr;  // [0] ordered: the x lines each unit's panels use (build_xmask)
    uint32_t rows_per_block = 0, nblocks = 0, npanels = 0, part_panels = 0, npad = 0, max_seg = 0, max_run = 0;
    uint64_t n_cont = 0;
    uint64_t ticket_words = 0, partial_bytes = 0;  // the combine scratch of one stream (split geometries)
    std::vector<uint32_t> block_first;  // nblocks + 1: first entry of each row block (last: nnz)
    int split = 1;
    bool row_runs = false;  // place_segments_banked: runs inside 16-lane rows (xlane 5 applies)
    bool vc4 = false;       // [2] built for k_vcache's four-part geometry (HIPSPMV_SPLIT4_VCACHE=1), not k_vquad
  } vc[5];  // [0] ordered (kVcOrdered), [1] split (kVcSplit); experimental: [2] split4; [3] wgather windows,
            // [4] wgather_split (kWgSplit)
  struct Vf {  // k_vflow layout (build_vflow), built on first selection ("kernel" VFLOW) or by AUTO
    bool ok = false, tried = false;
    uint32_t *d_code = nullptr, *d_wbeg = nullptr, *d_wend = nullptr, *d_tickets = nullptr;
    uint32_t* d_status = nullptr;  // bit 1: a flag wait gave up (the results of that launch are wrong)
    uint64_t *d_vals = nullptr, *d_partial = nullptr;
    uint32_t rows_per_block = 0, nblocks = 0, npanels = 0, part_panels = 0, npad = 0, max_group = 0;
    uint64_t ticket_words = 0, partial_bytes = 0;
    std::vector<uint32_t> block_first;  // nblocks + 1: first entry of each row block (last: nnz)
  } vf;
  int vflow_map = 0;  // option "vflow_map": 1 = XCDs 2h, 2h + 1 take column part h (vc_map.h MAP 1)
  int vflow_de = 4;   // option "vflow_de": steps of entries in flight per compute wave (2, 3, 4, 8)
  uint32_t* d_vfprof = nullptr;  // option "vflow_prof" (diagnostic): k_vflow's per-wave cycle stamps
  // The ordered vcache layout is only ever selected by name: its eligibility
  // and geometry are known at create, its entries built on first selection.
  bool vc0_eligible = false;
  // the four-part geometry's eligibility (create; the k_vquad layout itself is
  // built on first selection, ensure_layout, and may then prove unplaceable)
  bool vq_eligible = false;
  // k_wgather (x wider than the vcache geometries): eligibility and longest
  // in-window run measured at create; the layout is built at create when AUTO
  // picks the kernel, else on first selection by name
  bool wg_eligible = false;
  uint32_t wg_max_run = 0;
  bool wgs_eligible = false;  // the two-part form (kWgSplit): wgather-eligible, <= 2^21 rows
  struct Sell {  // k_sell layout: built at create when AUTO picks SELL, else on first selection
    bool built = false;
    uint64_t* d_off = nullptr;
    uint32_t *d_width = nullptr, *d_row = nullptr, *d_len = nullptr, *d_col = nullptr, *d_hubs = nullptr;
    uint32_t *d_pieces = nullptr, *d_tickets = nullptr;
    uint64_t *d_vals = nullptr, *d_partial = nullptr;
    uint32_t nslices = 0, nhubs = 0, npieces = 0, niso = 0, ntickets = 0;
    uint64_t padding = 0;
    std::vector<uint64_t> off;  // nslices + 1: first (padded) entry of each slice, on the host
  } sell;
  uint64_t wc_segments = 0;  // segments the wcsr layout would have (counted at create for wide x, else 0)
  struct Wc {  // wcsr: the column-windowed segment matrix (built when AUTO picks it, else on first selection)
    bool built = false;
    uint32_t *d_rowptr = nullptr, *d_colind = nullptr, *d_groups = nullptr, *d_rowseg = nullptr,
             *d_segidx = nullptr, *d_rgroups = nullptr, *d_chunks = nullptr;
    // the compact reduce (k_wreduce_c): rows with segments, their offsets, groups, the bitmap
    uint32_t *d_rrow = nullptr, *d_rsegc = nullptr, *d_cgroups = nullptr, *d_nebits = nullptr;
    uint32_t* d_hot = nullptr;  // hot-column form: [window][hotk] column ids staged in LDS (k_wpass_hot)
    uint32_t hotk = 0;
    uint64_t *d_vals = nullptr, *d_ypart = nullptr;
    uint32_t nseg = 0, ngroups = 0, rgroups = 0, ncgroups = 0, nrows_ne = 0, max_seg = 0, log2w = 0, nchunks = 0;
    std::vector<uint32_t> group_first;  // ngroups + 1: first entry of each segment-pass group (host)
  } wc;
  int vcache_dma = -1;   // option "vcache_dma": LDS-DMA x loader (-1 default: on for the split geometry)
  int vcache_xlane = -1;  // option "vcache_xlane": run continuation form (-1 default: cross-lane for split)
  int vcache_map = 0;    // option "vcache_map": XCD-aware part placement (unused since k_vquad; kept as an option)
  int vcache_xmask = 1;  // option "vcache_xmask": the ordered loaders skip unused x lines (0: load every line)
  int vquad_variant = 0;  // option "vquad_variant": k_vquad configuration (csrc/vquad.hip launch_vquad_t)
  // bit 0: reserved for a combine hand-off that timed out into unpublished
  // partials (csrc/combine.h has no such path since round 4; the word stays 0)
  uint32_t* d_status = nullptr;
  // hipspmv_attach_pmc: a rocprofv3 --pmc counter CSV whose counters back the
  // cache statistics read_misses / hazard_stalls / capacity_stalls
  std::string pmc_csv;
  // option "wgather_chunk": row blocks per k_wgather launch:
  // one launch's blocks are all resident at once (2 per CU), so they walk
  // the x windows together and the gathered window stays in L2
  uint32_t wgather_chunk = kWgChunk;
  // env HIPSPMV_WGATHER_SORT=0 at create: the wgather layout keeps (row, column) order in
  // each segment instead of sorting row runs by x line (probe)
  bool wgather_sort = true;
  // env HIPSPMV_WCSR_LINE=1 at create: wcsr segments by the x line of their
  // first column inside a window instead of by row (probe; C5 shards 2-7
  // measured 6 % slower)
  bool wcsr_line_order = false;
  // option "vcache_nt": row blocks b >= vcache_nt load their entries
  // non-temporally; -1 default: about kVcResidentBytes of
  // entries resident (resident_blocks; C3: half the blocks of either geometry)
  int64_t vcache_nt = -1;
  // option "wcsr_res": wcsr segment-pass groups g < wcsr_res load their entries
  // with the default policy (Infinity-Cache resident); 0 default: all non-temporal
  int64_t wcsr_res = 0;
  int wcsr_reduce = 0;    // option "wcsr_reduce": 0 the compact reduce over rows with segments, 1 every row
  int wcsr_xcd = 0;       // option "wcsr_xcd": 1 the segment pass's blocks placed by XCD eighths (kernels.hip)
  uint32_t wcsr_hot = 0;  // wcsr hot-column form: K (8192 / 16384) or 0 (HIPSPMV_WCSR_HOT at create)
  int wgather_map = 0;    // option "wgather_map": wgather_split's halves 0 by XCD, 1 alternating (diagnostic)
  int wcsr_fill = -1;     // option "wcsr_fill": 1 the rows without segments written by the segment pass's
                          // launch, 0 by the reduce's; -1 (default) 1 when two thirds of the rows are empty
  // option "sell_nt": SELL slices s >= sell_nt load their entries
  // non-temporally (-1 default: the second half of the slices)
  int64_t sell_nt = -1;
  int sell_only = 0;          // option "sell_only" (experimental timing probe)
  uint32_t sell_chain_g = 0;  // option "sell_chain" (experimental): ORDERED hub chain form (0 product)
  void *d_x = nullptr, *d_y = nullptr;
  int kernel_opt = HIPSPMV_KERNEL_AUTO, mode_opt = HIPSPMV_MODE_ORDERED, timing = 0;
  // setup_ns: create (transpose, validation, uploads, every layout AUTO uses);
  // layout_ns: layouts built later, on first selection by name (also counted
  // in the "setup_ns" statistic, so the plugin's setupTimeUs covers them)
  uint64_t setup_ns = 0, layout_ns = 0, kernel_ns = 0, h2d_ns = 0, d2h_ns = 0, execs = 0, device_bytes = 0;
  // create's phases: host CSR (copy or transpose, validation), CSR upload,
  // scans (eligibility, run and segment counts), layouts (build + upload)
  uint64_t setup_csr_ns = 0, setup_upload_ns = 0, setup_scan_ns = 0, setup_layouts_ns = 0;
  int auto_fallback = 0;  // AUTO layouts that could not be built (device OOM): the generic kernel runs instead
  int last_beta = 0;
  uint32_t max_row_len = 0, empty_rows = 0;
  int clock_khz = 0;  // shader clock (hipDeviceAttributeClockRate), for the cycle statistics
  int last_kernel = 0;
  // bytes of the last launch's entry stream loaded with the default cache policy (they may stay in
  // the Infinity Cache until the next launch; the rest load non-temporally): stat "resident_entry_bytes"
  uint64_t resident_entry_bytes = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool pending = false;  // kernel events recorded by exec_device, not yet read
  // The combine scratch (vcache_split/split4 tickets + partials, SELL FAST
  // hub-piece tickets + partials, wcsr segment partials) is one set per stream
  // (VERDICT r05 item 6): launches on different streams share none of it, so
  // the handle orders nothing across streams and records nothing on a
  // caller's stream -- a stream may be destroyed right after its last launch.
  // Set 0 is the layouts' own buffers, claimed by the first stream that
  // launches; sets 1.. are allocated on a stream's first launch of a kind
  // (zeroed on that stream, ahead of it).  Beyond kScratchSets streams the
  // least recently used set is taken over after a device synchronisation.
  // Streams are told apart by their handle value (hipStreamGetId is newer
  // than the HIP runtime PyTorch ships): a destroyed stream's value can come
  // back for a new stream only once the queue is gone, and HIP deletes a queue
  // after the work queued on it (hipStreamDestroy waits for it on ROCm --
  // checked by tests/test_gpu_streams.py), so a set is never shared by two
  // launches in flight.
  static constexpr int kScratchSets = 4;
  struct Scratch {
    bool assigned = false;
    uintptr_t sid = 0;  // the stream's handle value (NULL: the default stream)
    uint64_t last = 0;  // LRU tick
    uint32_t* vc_tickets[5] = {};  // per vc[] layout (split geometries: 1, 2, 4)
    uint64_t* vc_partial[5] = {};
    uint32_t* sell_tickets = nullptr;
    uint64_t* sell_partial = nullptr;
    uint64_t* wc_ypart = nullptr;
    uint32_t* vf_tickets = nullptr;
    uint64_t* vf_partial = nullptr;
  } scratch[kScratchSets];
  uint64_t scratch_tick = 0, scratch_evictions = 0;
  uint32_t* prof_tickets = nullptr;  // the tickets buffer the last profiled split launch stamped
  // option "profile" (DESIGN.md §6.9): vcache / vcache_split launches run with
  // the kernel's profile stamps; the NewCache state statistics come from them
  int profile = 0;
  uint32_t* d_prof = nullptr;  // ordered geometry: kVcProfWords per workgroup (split: inside d_tickets)
  bool prof_pending = false, prof_valid = false;
  hipStream_t prof_stream = nullptr;
  int prof_layout = 0;  // vc[] index of the profiled launch
  struct Prof {  // means over the workgroups of the last profiled launch, shader cycles
    uint64_t fill = 0, active = 0, flush = 0, done = 0, loader_work = 0, loader_wait = 0, compute_wait = 0;
    uint64_t units = 0, span = 0;
  } prof;
};

// Everything the handle owns on the device goes to the release thread
// (defer_release): the caller's thread does not wait for the device.
static void release(hipspmv_t* h) {
  if (!h) return;
  std::vector<void*> ptrs = {h->d_rowptr, h->d_colind, h->d_groups, h->d_vals, h->d_x, h->d_y, h->d_prof, h->d_status};
  for (auto& v : h->vc) ptrs.insert(ptrs.end(), {v.d_seg, v.d_code, v.d_tickets, v.d_vals, v.d_partial, v.d_xmask});
  {
    auto& q = h->sell;
    ptrs.insert(ptrs.end(), {q.d_off, q.d_width, q.d_row, q.d_len, q.d_col, q.d_hubs, q.d_vals, q.d_pieces,
                             q.d_tickets, q.d_partial});
  }
  {
    auto& w = h->wc;
    ptrs.insert(ptrs.end(), {w.d_rowptr, w.d_colind, w.d_groups, w.d_rowseg, w.d_segidx, w.d_rgroups, w.d_chunks,
                             w.d_vals, w.d_ypart, w.d_rrow, w.d_rsegc, w.d_cgroups, w.d_nebits, w.d_hot});
  }
  ptrs.push_back(h->d_vfprof);
  ptrs.insert(ptrs.end(), {h->vf.d_code, h->vf.d_wbeg, h->vf.d_wend, h->vf.d_tickets, h->vf.d_vals, h->vf.d_partial,
                           h->vf.d_status});
  for (int i = 1; i < hipspmv_handle::kScratchSets; ++i) {  // set 0 is the layouts' own (above)
    auto& c = h->scratch[i];
    for (int k = 0; k < 5; ++k) ptrs.insert(ptrs.end(), {c.vc_tickets[k], c.vc_partial[k]});
    ptrs.insert(ptrs.end(), {c.sell_tickets, c.sell_partial, c.wc_ypart, c.vf_tickets, c.vf_partial});
  }
  std::vector<void*> evs;
  for (hipEvent_t e : h->ev) evs.push_back(e);
  // HIPSPMV_SYNC_RELEASE=1 (diagnostic, tools/destroy_probe.py): the round-5 form, every buffer freed by
  // hipFree on the caller's thread -- the A/B that shows what a destroy inside a launch loop cost
  if (const char* sr = std::getenv("HIPSPMV_SYNC_RELEASE"); sr && std::strcmp(sr, "1") == 0) {
    DeviceGuard g(h->device);
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    for (void* e : evs)
      if (e) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return;
  }
  try {
    defer_release(h->device, std::move(ptrs), std::move(evs), {h->stream});
  } catch (...) {  // host OOM while queueing: the device memory leaks, nothing is freed under a live launch
  }
  delete h;
}

static void free_vc(hipspmv_t* h, int k) {
  auto& v = h->vc[k];
  void* vp[] = {v.d_seg, v.d_code, v.d_tickets, v.d_vals, v.d_partial, v.d_xmask};
  for (void* p : vp)
    if (p) (void)hipFree(p);
  v = hipspmv_handle::Vc{};
}

// Build vcache-family layout k (geometry g) from `a` and upload it; on
// failure nothing of it stays allocated.
static int upload_vc(hipspmv_t* h, int k, const HostCSR& a, const VcGeom& g, uint32_t lanes = 0) {
  auto& v = h->vc[k];
  const uint64_t bytes0 = h->device_bytes;
  VcacheLayout L;
  if (lanes) {  // k_vquad's placement (build_vcache_lanes); false: not placeable, not eligible
    if (!build_vcache_lanes(a, g, lanes, L)) return HIPSPMV_ERR_UNSUPPORTED;
  } else {
    build_vcache(a, g, L, (k == 3 || k == 4) && h->wgather_sort);  // k_wgather: gathers of one x line side by side
    // the vector-cache geometries (ordered and split): rows of each segment
    // placed for LDS banks (plan.cpp place_segments_banked; every row keeps its
    // run and its column order, so the sums are bit-identical);
    // HIPSPMV_VCACHE_BANK=0 keeps the (row, column) order (A/B probe)
    const char* bank = std::getenv("HIPSPMV_VCACHE_BANK");
    if ((k == 0 || k == 1 || (k == 2 && g.split == 4 && g.colbits == 16)) && !(bank && std::strcmp(bank, "0") == 0))
      place_segments_banked(L, k == 1 ? kVcSplitCT : k == 0 ? kVcOrderedCT : kVcSplit4CT);
  }
  v.split = g.split;
  v.rows_per_block = L.rows_per_block;
  v.nblocks = L.nblocks;
  v.npanels = L.npanels;
  v.part_panels = L.part_panels;
  v.npad = L.npad;
  v.max_seg = L.max_seg;
  v.max_run = L.max_run;
  v.n_cont = L.n_cont;
  v.row_runs = L.row_runs;
  v.block_first.assign(L.nblocks + 1, (uint32_t)L.code.size());
  for (uint32_t b = 0; b < L.nblocks; ++b) v.block_first[b] = L.seg[(size_t)b * L.geom.split * (L.npad + 1)];
  auto fail = [&](int st) {
    free_vc(h, k);
    h->device_bytes = bytes0;
    return st;
  };
  int st;
  if ((st = dev_upload(&v.d_seg, L.seg.data(), L.seg.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&v.d_code, L.code.data(), L.code.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&v.d_vals, L.vals.data(), L.vals.size(), h->device_bytes))) return fail(st);
  if (k == 0) {  // the ordered geometry's loaders skip the x lines no entry of a panel uses
    std::vector<uint64_t> xm;
    build_xmask(L, kVcOrderedLoaders, xm);
    if ((st = dev_upload(&v.d_xmask, xm.data(), xm.size(), h->device_bytes))) return fail(st);
  }
  if (v.split > 1) {
    // [4 b, 4 b + split): the published-share counters of block b (the owner
    // combine, csrc/combine.h; they return to 0 within each launch), then
    // kVcProfWords per unit for the profile stamps (option "profile")
    std::vector<uint32_t> zeros(4ull * v.nblocks + (uint64_t)kVcProfWords * v.nblocks * v.split, 0u);
    if ((st = dev_upload(&v.d_tickets, zeros.data(), zeros.size(), h->device_bytes))) return fail(st);
    // partials: part q of block b at (q * nblocks + b) * VRP doubles, VRP = the
    // geometry's y block rounded up to even (k_vcache's 16-byte combine)
    const uint64_t pbytes = 8ull * v.split * v.nblocks * (((uint32_t)g.rows + 1) & ~1u);
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&v.d_partial), pbytes);
    if (e != hipSuccess) return fail(hip_fail(e, "hipMalloc(partials)"));
    h->device_bytes += pbytes;
    v.ticket_words = zeros.size();
    v.partial_bytes = pbytes;
  }
  v.ok = true;
  return HIPSPMV_OK;
}

// Frees whatever a layout build that threw (host std::bad_alloc) had already
// uploaded: the half-built SELL / wcsr / vcache-family layouts, so a later
// build starts from nothing and nothing stays allocated behind a failed one.
static void drop_partial_layouts(hipspmv_t* h) {
  DeviceGuard g(h->device);
  if (!h->sell.built) {
    auto& q = h->sell;
    void* sp[] = {q.d_off, q.d_width, q.d_row, q.d_len, q.d_col, q.d_hubs, q.d_vals, q.d_pieces, q.d_tickets,
                  q.d_partial};
    for (void* p : sp)
      if (p) (void)hipFree(p);
    q = hipspmv_handle::Sell{};
  }
  if (!h->wc.built) {
    auto& w = h->wc;
    void* wp[] = {w.d_rowptr, w.d_colind, w.d_groups, w.d_rowseg, w.d_segidx, w.d_rgroups, w.d_chunks, w.d_vals, w.d_ypart,
                  w.d_rrow, w.d_rsegc, w.d_cgroups, w.d_nebits, w.d_hot};
    for (void* p : wp)
      if (p) (void)hipFree(p);
    w = hipspmv_handle::Wc{};
  }
  for (int k = 0; k < 5; ++k)
    if (!h->vc[k].ok && (h->vc[k].d_seg || h->vc[k].d_code || h->vc[k].d_vals)) {
      const auto keep = h->vc[k];  // the ordered geometry is known before its entries exist
      free_vc(h, k);
      h->vc[k].split = keep.split;
      h->vc[k].rows_per_block = keep.rows_per_block;
      h->vc[k].nblocks = keep.nblocks;
      h->vc[k].npanels = keep.npanels;
      h->vc[k].part_panels = keep.part_panels;
      h->vc[k].npad = keep.npad;
      h->vc[k].max_run = keep.max_run;
    }
}

// The device CSR copy back on the host (the host CSR is gone after create):
// the source of the layouts built on first selection by name.
static int download_csr(hipspmv_t* h, HostCSR& a) {
  a.rows = h->rows;
  a.cols = h->cols;
  a.nnz = h->nnz;
  a.rowptr.resize((size_t)h->rows + 1);
  a.colind.resize(h->nnz);
  a.vals.resize(h->nnz);
  HIP_TRY(hipMemcpy(a.rowptr.data(), h->d_rowptr, 4ull * (h->rows + 1), hipMemcpyDeviceToHost));
  if (h->nnz) {
    HIP_TRY(hipMemcpy(a.colind.data(), h->d_colind, 4ull * h->nnz, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(a.vals.data(), h->d_vals, 8ull * h->nnz, hipMemcpyDeviceToHost));
  }
  return HIPSPMV_OK;
}

// The SELL layout from the CSR `a`.
static int build_sell_layout(hipspmv_t* h, const HostCSR& a) {
  auto& q = h->sell;
  if (q.built) return HIPSPMV_OK;
  DeviceGuard g(h->device);
  SellLayout L;
  build_sell(a, L);
  const uint64_t bytes0 = h->device_bytes;
  auto fail = [&](int st) {  // a later attempt starts from nothing
    void* sp[] = {q.d_off, q.d_width, q.d_row, q.d_len, q.d_col, q.d_hubs, q.d_vals, q.d_pieces, q.d_tickets,
                  q.d_partial};
    for (void* p : sp)
      if (p) (void)hipFree(p);
    q = hipspmv_handle::Sell{};
    h->device_bytes = bytes0;
    return st;
  };
  int st;
  if ((st = dev_upload(&q.d_off, L.off.data(), L.off.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_width, L.width.data(), L.width.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_row, L.row.data(), L.row.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_len, L.len.data(), L.len.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_col, L.col.data(), L.col.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_vals, L.vals.data(), L.vals.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_hubs, L.hubs.data(), L.hubs.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&q.d_pieces, L.pieces.data(), L.pieces.size(), h->device_bytes))) return fail(st);
  {
    const std::vector<uint32_t> zeros(L.ntickets, 0u);  // tickets self-reset after each launch
    if ((st = dev_upload(&q.d_tickets, zeros.data(), zeros.size(), h->device_bytes))) return fail(st);
    const std::vector<uint64_t> none(L.npieces, 0u);
    if ((st = dev_upload(&q.d_partial, none.data(), none.size(), h->device_bytes))) return fail(st);
  }
  q.npieces = L.npieces;
  q.ntickets = L.ntickets;
  q.off = L.off;
  q.nslices = L.nslices;
  q.nhubs = L.nhubs;
  q.niso = L.niso;
  q.padding = L.padding;
  q.built = true;
  return HIPSPMV_OK;
}

// The wcsr layout (column-windowed segment matrix) from the CSR `a`.
static int build_wcsr_layout(hipspmv_t* h, const HostCSR& a) {
  auto& w = h->wc;
  if (w.built) return HIPSPMV_OK;
  DeviceGuard g(h->device);
  // the global-x form (windows of 2^kWcLog2Window), or with HIPSPMV_WCSR_LDS=1
  // the LDS form (k_wseg: x windows of 2^kWsLog2Window staged in LDS; slower
  // on every C5 shard measured)
  const char* lds_env = std::getenv("HIPSPMV_WCSR_LDS");
  const bool lds = lds_env && std::strcmp(lds_env, "1") == 0;
  // windows of 2^kWcLog2Window columns for every matrix (a width that does
  // not depend on the matrix keeps a row's segments the same in every row
  // partition of it)
  uint32_t log2w = lds ? kWsLog2Window : kWcLog2Window;
  if (const char* e = std::getenv("HIPSPMV_WCSR_LOG2W"); e && !lds) {  // probe: another window width
    const int v = std::atoi(e);
    if (v >= 10 && v <= 24) log2w = (uint32_t)v;
  }
  // segments of at most kCvGroupNnz entries, so every segment-pass group is a
  // balanced multi-row group (C5 shard 0 / 3: 264.1 / 314.2 -> 257.2 / 306.5
  // us); HIPSPMV_WCSR_MAXSEG overrides (probe)
  uint32_t cap = (uint32_t)kCvGroupNnz;
  if (const char* e = std::getenv("HIPSPMV_WCSR_MAXSEG")) cap = (uint32_t)std::max(64, std::atoi(e));
  WinLayout L;
  build_windowed(a, log2w, L, cap, !lds && h->wcsr_line_order);
  // the hot-column form (kernels.hip k_wpass_hot): each window's K most frequent columns staged in
  // LDS by every segment-pass workgroup (HIPSPMV_WCSR_HOT=K at create: 8192 or 16384; 0 off)
  uint32_t hotk = h->wcsr_hot;
  if (const char* e = std::getenv("HIPSPMV_WCSR_HOT")) hotk = (uint32_t)std::max(0, std::atoi(e));
  if (!kExperimental) hotk = 0;  // measured slower: experimental build only
  if (hotk != 8192 && hotk != kWcHotMax) hotk = 0;
  std::vector<uint32_t> hot;
  if (lds || !hotk || !mark_hot_columns(L, hotk, hot)) {  // (the remap runs only for a hot layout)
    hotk = 0;
    hot.clear();
  }
  std::vector<uint32_t> groups, chunks;
  if (lds || hotk) {  // csr_vector groups inside each window, cut into chunks of <= kWsChunkNnz entries
    // (hot form: chunks of about nnz / 240 entries -- one wave of 1024-thread workgroups over the chip,
    // each staging its window's hot columns once)
    // (8192 hot columns: 64 KiB of LDS, two workgroups per CU -- twice the chunks)
    const uint32_t chunk_nnz =
        lds ? kWsChunkNnz : std::max<uint32_t>(8192u, (uint32_t)(a.nnz / (hotk == kWcHotMax ? 240u : 480u) + 1));
    const auto& rp = L.seg.rowptr;
    for (uint32_t win = 0; win + 1 < L.winseg.size(); ++win) {
      const uint32_t s0 = L.winseg[win], s1 = L.winseg[win + 1];
      if (s0 == s1) continue;
      std::vector<uint32_t> wg;
      build_row_groups(rp.data() + s0, s1 - s0, wg);
      uint32_t cg = (uint32_t)groups.size(), cnnz = 0;
      for (size_t i = 0; i + 1 < wg.size(); ++i) {
        const uint32_t n = rp[s0 + wg[i + 1]] - rp[s0 + wg[i]];
        if (cnnz && cnnz + n > chunk_nnz) {
          chunks.insert(chunks.end(), {win, cg, (uint32_t)groups.size()});
          cg = (uint32_t)groups.size();
          cnnz = 0;
        }
        groups.push_back(s0 + wg[i]);
        cnnz += n;
      }
      chunks.insert(chunks.end(), {win, cg, (uint32_t)groups.size()});
    }
    groups.push_back(L.nseg);
  } else {
    build_row_groups(L.seg, groups);
  }
  const uint64_t bytes0 = h->device_bytes;
  auto fail = [&](int st) {
    void* wp[] = {w.d_rowptr, w.d_colind, w.d_groups, w.d_rowseg, w.d_segidx, w.d_rgroups, w.d_chunks,
                  w.d_vals, w.d_ypart, w.d_rrow, w.d_rsegc, w.d_cgroups, w.d_nebits, w.d_hot};
    for (void* p : wp)
      if (p) (void)hipFree(p);
    w = hipspmv_handle::Wc{};
    h->device_bytes = bytes0;
    return st;
  };
  int st;
  if ((st = dev_upload(&w.d_rowptr, L.seg.rowptr.data(), L.seg.rowptr.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&w.d_colind, L.seg.colind.data(), L.seg.colind.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&w.d_vals, L.seg.vals.data(), L.seg.vals.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&w.d_groups, groups.data(), groups.size(), h->device_bytes))) return fail(st);
  if (!chunks.empty() && (st = dev_upload(&w.d_chunks, chunks.data(), chunks.size(), h->device_bytes)))
    return fail(st);
  w.nchunks = (uint32_t)(chunks.size() / 3);
  if (hotk && (st = dev_upload(&w.d_hot, hot.data(), hot.size(), h->device_bytes))) return fail(st);
  w.hotk = hotk;
  if ((st = dev_upload(&w.d_rowseg, L.rowseg.data(), L.rowseg.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&w.d_segidx, L.segidx.data(), L.segidx.size(), h->device_bytes))) return fail(st);
  {  // the reduce is a csr_vector over (rowseg, segidx) with ypart as x: its own balanced row groups
    std::vector<uint32_t> rg;
    build_row_groups(L.rowseg.data(), a.rows, rg);
    if ((st = dev_upload(&w.d_rgroups, rg.data(), rg.size(), h->device_bytes))) return fail(st);
    w.rgroups = (uint32_t)rg.size() - 1;
  }
  {  // the compact reduce: the rows with segments, in order, and a bitmap of them for the fill
    std::vector<uint32_t> rrow, rsegc, cg, bits(((size_t)a.rows + 31) / 32, 0u);
    for (uint32_t r = 0; r < a.rows; ++r)
      if (L.rowseg[r + 1] > L.rowseg[r]) {
        rrow.push_back(r);
        rsegc.push_back(L.rowseg[r]);
        bits[r >> 5] |= 1u << (r & 31);
      }
    rsegc.push_back(L.rowseg[a.rows]);
    build_row_groups(rsegc.data(), (uint32_t)rrow.size(), cg);
    if (!rrow.empty() && (st = dev_upload(&w.d_rrow, rrow.data(), rrow.size(), h->device_bytes))) return fail(st);
    if ((st = dev_upload(&w.d_rsegc, rsegc.data(), rsegc.size(), h->device_bytes))) return fail(st);
    if ((st = dev_upload(&w.d_cgroups, cg.data(), cg.size(), h->device_bytes))) return fail(st);
    if (!bits.empty() && (st = dev_upload(&w.d_nebits, bits.data(), bits.size(), h->device_bytes))) return fail(st);
    w.ncgroups = (uint32_t)cg.size() - 1;
    w.nrows_ne = (uint32_t)rrow.size();
  }
  {
    const uint64_t b = 8ull * std::max<uint32_t>(L.nseg, 1);
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&w.d_ypart), b);
    if (e != hipSuccess) return fail(hip_fail(e, "hipMalloc(segment partials)"));
    h->device_bytes += b;
  }
  w.nseg = L.nseg;
  w.ngroups = (uint32_t)groups.size() - 1;
  w.group_first.resize(groups.size());
  for (size_t g = 0; g < groups.size(); ++g) w.group_first[g] = L.seg.rowptr[groups[g]];
  w.max_seg = L.max_seg;
  w.log2w = L.log2w;
  w.built = true;
  return HIPSPMV_OK;
}

// The vcache-family layout k from the CSR `a` (k 0: ordered vcache, 3: wgather, 4: wgather_split).
static int build_vc_layout(hipspmv_t* h, int k, const HostCSR& a) {
  if (h->vc[k].ok) return HIPSPMV_OK;
  if (k == 0 && !h->vc0_eligible) return HIPSPMV_ERR_UNSUPPORTED;
  if (k == 3 && !h->wg_eligible) return HIPSPMV_ERR_UNSUPPORTED;
  if (k == 4 && !h->wgs_eligible) return HIPSPMV_ERR_UNSUPPORTED;
  DeviceGuard g(h->device);
  return upload_vc(h, k, a, k == 0 ? kVcOrdered : k == 3 ? kWgWindow : kWgSplit);
}

// AUTO, from the round-2 sweeps on MI355X:
//  * the LDS vector cache pays when each x element a work unit streams
//    feeds enough nonzeros and no row runs long inside a segment (C3 FAST:
//    vcache_split 124 us);
//  * x wider than the vcache geometries, short runs: the windowed gather
//    (2^21 x 2^24 stripe shard: wgather 455 us vs sell 1070, csr_vector 1297);
//  * otherwise ORDERED takes SELL (C3: 199 us vs vcache 217, csr_lane 1453;
//    R-MAT s20: 527 us vs csr_lane 12136) and FAST csr_vector (R-MAT s20:
//    253 us vs sell 573, vcache_split 23572) unless one row outlasts the
//    rest (below).
// `built`: only kernels whose layout exists (the exec paths); false: what
// AUTO wants (create, which then builds those layouts).  A wanted layout that
// could not be built falls back to the generic kernel of the mode: csr_lane
// (ORDERED) or csr_vector (FAST), which need nothing beyond the CSR copy.
static int auto_pick(const hipspmv_t* h, bool fast_ok, bool built) {
  // each x element a work unit streams feeds enough nonzeros (geometry only:
  // the ordered layout's entries are built once AUTO wants them)
  auto worth = [&](const hipspmv_handle::Vc& v, bool eligible) {
    return eligible && v.max_run <= kVcRunMax &&
           (uint64_t)h->nnz * 16 * v.split >= (uint64_t)v.nblocks * v.split * h->cols;
  };
  const int generic = fast_ok ? HIPSPMV_KERNEL_CSR_VECTOR : HIPSPMV_KERNEL_CSR_LANE;
  if (fast_ok && worth(h->vc[1], h->vc[1].ok)) return HIPSPMV_KERNEL_VCACHE_SPLIT;
  // ORDERED: the ordered vector cache with half its row blocks' entries
  // non-temporal (C3: 181 us against sell's 185 with the same policy, 199 as
  // round 2 ran it)
  if (!fast_ok && worth(h->vc[0], h->vc0_eligible))
    return !built || h->vc[0].ok ? HIPSPMV_KERNEL_VCACHE : h->sell.built ? HIPSPMV_KERNEL_SELL : generic;
  // FAST with at most 2^21 rows (a C4 shard): the two-part form, 16384-row
  // blocks, each XCD's L2 holding half of x (2^21 x 2^24 stripe shard:
  // DESIGN.md §6.18)
  if (fast_ok && !h->vc0_eligible && h->wgs_eligible && h->wg_max_run <= kVcRunMax)
    return !built || h->vc[4].ok ? HIPSPMV_KERNEL_WGATHER_SPLIT : generic;
  if (!h->vc0_eligible && h->wg_eligible && h->wg_max_run <= kVcRunMax)
    return !built || h->vc[3].ok ? HIPSPMV_KERNEL_WGATHER : generic;
  if (!fast_ok) return !built || h->sell.built ? HIPSPMV_KERNEL_SELL : generic;
  // csr_vector gives a long row one wave (256 entries per ~1.6 us step): when
  // that row alone outlasts the bulk of the matrix (~1 TB/s of algorithmic
  // bytes), SELL's FAST hub pieces spread it over many waves.  C5 shard 0 of 8
  // (70 k hub rows, longest 238 k): csr_vector 2019 us, sell 496 us; R-MAT s20
  // (longest 39.7 k): csr_vector 253 us, sell 573 us.
  // x wider than the L2s and rows that keep several entries per column window:
  // csr_vector over the windowed segments (C5 shards 0 / 7 of 8: 238 / 280 us
  // against sell 479 / csr_vector 628); C4's uniform rows
  // (one entry per window) stay on wgather above
  if (h->wc_segments && h->wc_segments * 2 <= h->nnz) return !built || h->wc.built ? HIPSPMV_KERNEL_WCSR : generic;
  const uint64_t alg = 12ull * h->nnz + 4ull * (h->rows + 1ull) + 8ull * h->cols + 8ull * h->rows;
  if ((uint64_t)h->max_row_len * 4167ull > alg) return !built || h->sell.built ? HIPSPMV_KERNEL_SELL : generic;
  return HIPSPMV_KERNEL_CSR_VECTOR;
}

static int finish_create(hipspmv_t* h, HostCSR& a) {
  DeviceGuard g(h->device);
  HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  for (auto& e : h->ev) HIP_TRY(hipEventCreate(&e));
  for (uint32_t r = 0; r < a.rows; ++r) {
    const uint32_t len = a.rowptr[r + 1] - a.rowptr[r];
    h->max_row_len = len > h->max_row_len ? len : h->max_row_len;
    h->empty_rows += len == 0;
  }
  int st;
  uint64_t t0 = now_ns();
  if ((st = dev_upload(&h->d_rowptr, a.rowptr.data(), a.rowptr.size(), h->device_bytes))) return st;
  if ((st = dev_upload(&h->d_colind, a.colind.data(), a.colind.size(), h->device_bytes))) return st;
  if ((st = dev_upload(&h->d_vals, a.vals.data(), a.vals.size(), h->device_bytes))) return st;
  std::vector<uint32_t> groups;
  build_row_groups(a, groups);
  h->ngroups = (uint32_t)groups.size() - 1;
  if ((st = dev_upload(&h->d_groups, groups.data(), groups.size(), h->device_bytes))) return st;
  h->setup_upload_ns = now_ns() - t0;
  t0 = now_ns();
  // experimental builds (HIPSPMV_EXPERIMENTAL=1) also build the wgather
  // window layout at create (below)
  const char* exp = std::getenv("HIPSPMV_EXPERIMENTAL");
  const bool experimental = exp && std::strcmp(exp, "1") == 0;
  // ordered vcache: geometry now, entries on first selection by name
  h->vc0_eligible = vcache_eligible(a, kVcOrdered);
  if (h->vc0_eligible) {
    VcacheLayout G;
    vcache_geometry(a.rows, a.cols, kVcOrdered, G);
    auto& v = h->vc[0];
    v.split = 1;
    v.rows_per_block = G.rows_per_block;
    v.nblocks = G.nblocks;
    v.npanels = G.npanels;
    v.part_panels = G.part_panels;
    v.npad = G.npad;
    v.max_run = vcache_max_run(a, (uint32_t)kVcOrdered.panel);
  }
  {
    const uint32_t zero = 0;
    if ((st = dev_upload(&h->d_status, &zero, 1, h->device_bytes))) return st;
  }
  const bool split_ok = vcache_eligible(a, kVcSplit), quad_ok = vcache_eligible(a, kVcQuad);
  h->wg_eligible = vcache_eligible(a, kWgWindow);
  if (h->wg_eligible) h->wg_max_run = vcache_max_run(a, (uint32_t)kWgWindow.panel);
  // (probe HIPSPMV_WGS_MAXROWS: another row cap for the two-part form, for its A/B on larger shards)
  uint64_t wgs_cap = 128ull * (uint32_t)kWgSplit.rows;
  if (const char* e = std::getenv("HIPSPMV_WGS_MAXROWS")) wgs_cap = std::strtoull(e, nullptr, 10);
  h->wgs_eligible = h->wg_eligible && a.rows <= wgs_cap && vcache_eligible(a, kWgSplit);
  if (a.cols >= kWcMinCols) h->wc_segments = windowed_segments(a, kWcLog2Window);
  h->setup_scan_ns = now_ns() - t0;
  t0 = now_ns();
  if (split_ok && (st = upload_vc(h, 1, a, kVcSplit))) return st;
  // the four-part layout (k_vquad, never chosen by AUTO) is built on first
  // selection by name (ensure_layout), like the ordered vcache's
  h->vq_eligible = quad_ok;
  // the layouts AUTO will run, built now from the host CSR (no copy back off
  // the device at first use, and their time is setup time); device OOM here
  // leaves AUTO on the generic kernels instead of failing the create
  const bool exact_any = h->dtype == HIPSPMV_U64;
  for (const bool fast_ok : {exact_any, true}) {
    const int k = auto_pick(h, fast_ok, false);
    try {  // a host allocation failure in a layout build is an OOM like a device one
      if (k == HIPSPMV_KERNEL_SELL) st = build_sell_layout(h, a);
      else if (k == HIPSPMV_KERNEL_WGATHER) st = build_vc_layout(h, 3, a);
      else if (k == HIPSPMV_KERNEL_WGATHER_SPLIT) st = build_vc_layout(h, 4, a);
      else if (k == HIPSPMV_KERNEL_VCACHE) st = build_vc_layout(h, 0, a);
      else if (k == HIPSPMV_KERNEL_WCSR) st = build_wcsr_layout(h, a);
      else st = HIPSPMV_OK;
    } catch (const std::bad_alloc&) {
      drop_partial_layouts(h);
      st = HIPSPMV_ERR_OOM;
    }
    if (st == HIPSPMV_ERR_OOM) {
      h->auto_fallback++;
      (void)hipGetLastError();  // the failed allocation must not leak into a later check
    } else if (st) {
      return st;
    }
  }
  if (experimental && h->wg_eligible && (st = build_vc_layout(h, 3, a))) return st;
  h->setup_layouts_ns = now_ns() - t0;
  return HIPSPMV_OK;
}

template <typename Build>
static int create_common(uint32_t rows, uint32_t cols, uint32_t nnz, int dtype, int device, hipspmv_t** out,
                         Build build) {
  if (!out) return HIPSPMV_ERR_INVALID_ARG;
  *out = nullptr;
  if (dtype != HIPSPMV_F64 && dtype != HIPSPMV_U64) return HIPSPMV_ERR_INVALID_ARG;
  if (rows == 0 || cols == 0) return HIPSPMV_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_last_error = "no HIP device";
    return HIPSPMV_ERR_NO_DEVICE;
  }
  if (device < 0 || device >= ndev) return HIPSPMV_ERR_NO_DEVICE;
  const uint64_t t0 = now_ns();
  HostCSR a;
  std::string why;
  int st = build(a, why);
  if (st) {
    g_last_error = why;
    return st;
  }
  const uint64_t csr_ns = now_ns() - t0;
  hipspmv_t* h = new hipspmv_t;
  h->device = device;
  h->dtype = dtype;
  if (const char* e = std::getenv("HIPSPMV_WGATHER_SORT")) h->wgather_sort = std::strcmp(e, "0") != 0;
  if (const char* e = std::getenv("HIPSPMV_WCSR_LINE")) h->wcsr_line_order = std::strcmp(e, "1") == 0;
  h->rows = rows;
  h->cols = cols;
  h->nnz = nnz;
  h->setup_csr_ns = csr_ns;
  if (hipDeviceGetAttribute(&h->clock_khz, hipDeviceAttributeClockRate, device) != hipSuccess) h->clock_khz = 0;
  try {
    st = finish_create(h, a);
  } catch (...) {  // nothing uploaded so far may leak past a throw
    release(h);
    throw;
  }
  if (st) {
    release(h);
    return st;
  }
  h->setup_ns = now_ns() - t0;
  *out = h;
  return HIPSPMV_OK;
}

// Which kernel runs for `mode` (HIPSPMV_KERNEL_*), or a negative status.
static int choose_kernel(const hipspmv_t* h, int mode) {
  if (mode == HIPSPMV_MODE_AUTO) mode = h->mode_opt;
  if (mode != HIPSPMV_MODE_ORDERED && mode != HIPSPMV_MODE_FAST) return -HIPSPMV_ERR_INVALID_ARG;
  const bool exact_any = h->dtype == HIPSPMV_U64;  // integer sums are order-independent
  const bool fast_ok = mode == HIPSPMV_MODE_FAST || exact_any;
  switch (h->kernel_opt) {
    case HIPSPMV_KERNEL_VCACHE:  // layout built on first selection
      return h->vc0_eligible ? HIPSPMV_KERNEL_VCACHE : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_VCACHE_SPLIT:
      if (!fast_ok) return -HIPSPMV_ERR_UNSUPPORTED;
      return h->vc[1].ok ? HIPSPMV_KERNEL_VCACHE_SPLIT : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_VCACHE_SPLIT4:
      if (!fast_ok) return -HIPSPMV_ERR_UNSUPPORTED;
      return h->vc[2].ok || h->vq_eligible ? HIPSPMV_KERNEL_VCACHE_SPLIT4 : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_WGATHER:  // ordered: valid in both modes
      return h->vc[3].ok || h->wg_eligible ? HIPSPMV_KERNEL_WGATHER : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_WGATHER_SPLIT:
      if (!fast_ok) return -HIPSPMV_ERR_UNSUPPORTED;
      return h->vc[4].ok || h->wgs_eligible ? HIPSPMV_KERNEL_WGATHER_SPLIT : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_CSR_LANE:
      return HIPSPMV_KERNEL_CSR_LANE;
    case HIPSPMV_KERNEL_SELL:  // ordered: valid in both modes
      return HIPSPMV_KERNEL_SELL;
    case HIPSPMV_KERNEL_WCSR:  // fast; any matrix, layout built on first selection
      return fast_ok ? HIPSPMV_KERNEL_WCSR : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_CSR_VECTOR:
      return fast_ok ? HIPSPMV_KERNEL_CSR_VECTOR : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_VCACHE_FLOW:  // fast; layout built on first selection (may prove not eligible)
      if (!fast_ok) return -HIPSPMV_ERR_UNSUPPORTED;
      return h->vf.ok || !h->vf.tried ? HIPSPMV_KERNEL_VCACHE_FLOW : -HIPSPMV_ERR_UNSUPPORTED;
    case HIPSPMV_KERNEL_AUTO:
      return auto_pick(h, fast_ok, true);
    default:
      return -HIPSPMV_ERR_INVALID_ARG;
  }
}

// The layout a kernel selected by name needs, built on its first selection
// from the device CSR copy (AUTO's layouts exist since create); the time is
// added to the handle's setup time.
// The k_vflow layout from the CSR `a` (build_vflow); HIPSPMV_ERR_UNSUPPORTED
// when the matrix does not fit it (then never tried again).
static int build_vflow_layout(hipspmv_t* h, const HostCSR& a) {
  auto& f = h->vf;
  if (f.ok) return HIPSPMV_OK;
  if (f.tried) return HIPSPMV_ERR_UNSUPPORTED;
  f.tried = true;
  VflowLayout V;
  if (!build_vflow(a, V)) return HIPSPMV_ERR_UNSUPPORTED;
  const VcacheLayout& L = V.L;
  DeviceGuard g(h->device);
  const uint64_t bytes0 = h->device_bytes;
  auto fail = [&](int st) {
    void* fp[] = {f.d_code, f.d_wbeg, f.d_wend, f.d_tickets, f.d_vals, f.d_partial, f.d_status};
    for (void* p : fp)
      if (p) (void)hipFree(p);
    f = hipspmv_handle::Vf{};
    f.tried = true;
    h->device_bytes = bytes0;
    return st;
  };
  int st;
  if ((st = dev_upload(&f.d_code, L.code.data(), L.code.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&f.d_vals, L.vals.data(), L.vals.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&f.d_wbeg, V.wbeg.data(), V.wbeg.size(), h->device_bytes))) return fail(st);
  if ((st = dev_upload(&f.d_wend, V.wend.data(), V.wend.size(), h->device_bytes))) return fail(st);
  const std::vector<uint32_t> zeros(4ull * L.nblocks, 0u);  // owner-combine share counters
  if ((st = dev_upload(&f.d_tickets, zeros.data(), zeros.size(), h->device_bytes))) return fail(st);
  const uint64_t pbytes = 8ull * kVfGeom.split * L.nblocks * (uint32_t)kVfGeom.rows;
  const hipError_t e = hipMalloc(reinterpret_cast<void**>(&f.d_partial), pbytes);
  if (e != hipSuccess) return fail(hip_fail(e, "hipMalloc(vflow partials)"));
  h->device_bytes += pbytes;
  {
    const uint32_t z = 0;
    if ((st = dev_upload(&f.d_status, &z, 1, h->device_bytes))) return fail(st);
  }
  f.rows_per_block = L.rows_per_block;
  f.nblocks = L.nblocks;
  f.npanels = L.npanels;
  f.part_panels = L.part_panels;
  f.npad = L.npad;
  f.max_group = V.max_group;
  f.ticket_words = zeros.size();
  f.partial_bytes = pbytes;
  f.block_first.assign(L.nblocks + 1, (uint32_t)L.code.size());
  for (uint32_t b = 0; b < L.nblocks; ++b) f.block_first[b] = L.seg[(size_t)b * kVfGeom.split * (L.npad + 1)];
  f.ok = true;
  return HIPSPMV_OK;
}

static int ensure_layout(hipspmv_t* h, int kernel) {
  const bool need = (kernel == HIPSPMV_KERNEL_SELL && !h->sell.built) ||
                    (kernel == HIPSPMV_KERNEL_WGATHER && !h->vc[3].ok) ||
                    (kernel == HIPSPMV_KERNEL_WGATHER_SPLIT && !h->vc[4].ok) ||
                    (kernel == HIPSPMV_KERNEL_VCACHE && !h->vc[0].ok) ||
                    (kernel == HIPSPMV_KERNEL_VCACHE_SPLIT4 && !h->vc[2].ok) ||
                    (kernel == HIPSPMV_KERNEL_WCSR && !h->wc.built) ||
                    (kernel == HIPSPMV_KERNEL_VCACHE_FLOW && !h->vf.ok);
  if (!need) return HIPSPMV_OK;
  const uint64_t t0 = now_ns();
  int st;
  try {
    DeviceGuard g(h->device);
    HostCSR a;
    st = download_csr(h, a);
    if (!st) {
      if (kernel == HIPSPMV_KERNEL_SELL) st = build_sell_layout(h, a);
      else if (kernel == HIPSPMV_KERNEL_WCSR) st = build_wcsr_layout(h, a);
      else if (kernel == HIPSPMV_KERNEL_VCACHE_FLOW) st = build_vflow_layout(h, a);
      else if (kernel == HIPSPMV_KERNEL_VCACHE_SPLIT4) {
        // every segment inside the kernel's register window, runs placeable
        // (build_vcache_lanes); otherwise not eligible from now on
        // HIPSPMV_SPLIT4_VCACHE=1 (probe): the k_vcache four-part geometry with banked segments instead
        const char* v4 = std::getenv("HIPSPMV_SPLIT4_VCACHE");
        const bool vc4 = v4 && std::strcmp(v4, "1") == 0;
        st = !h->vq_eligible ? HIPSPMV_ERR_UNSUPPORTED
             : vc4 ? (vcache_eligible(a, kVcSplit4) ? upload_vc(h, 2, a, kVcSplit4) : HIPSPMV_ERR_UNSUPPORTED)
                   : upload_vc(h, 2, a, kVcQuad, kVqLanes);
        if (!st) h->vc[2].vc4 = vc4;
        if (st == HIPSPMV_ERR_UNSUPPORTED) h->vq_eligible = false;
      } else st = build_vc_layout(h, kernel == HIPSPMV_KERNEL_WGATHER ? 3 : kernel == HIPSPMV_KERNEL_WGATHER_SPLIT ? 4 : 0, a);
    }
  } catch (const std::bad_alloc&) {
    drop_partial_layouts(h);
    st = HIPSPMV_ERR_OOM;
  } catch (...) {  // e.g. std::system_error from the layout builder's threads
    drop_partial_layouts(h);
    g_last_error = "layout build failed";
    st = HIPSPMV_ERR_HIP;
  }
  h->layout_ns += now_ns() - t0;
  return st;
}

// Row blocks of a vcache layout whose entries load with the default cache
// policy, so they stay in the 256 MiB Infinity Cache from one launch to the
// next; the rest load non-temporally (nt lines do not displace resident ones,
// DESIGN.md §6.10).  About kVcResidentBytes of entries stay resident: C3 (384
// MiB of entries) keeps half its blocks -- split 101.9 -> 98.0 us, ordered
// 179 -> 168 us with the banked layouts; more starves x of L2
// and MALL (5/8: 102.6 us).
static uint32_t resident_blocks(uint32_t nblocks, uint64_t nnz) {
  const double entry_bytes = 12.0 * (double)nnz;
  if (entry_bytes <= (double)kVcResidentBytes) return nblocks;
  return (uint32_t)((double)nblocks * (double)kVcResidentBytes / entry_bytes);
}

// Set 0 of the combine scratch: the buffers the layouts allocated.
static void scratch_set0(hipspmv_t* h) {
  auto& c = h->scratch[0];
  for (int k = 0; k < 5; ++k) {
    c.vc_tickets[k] = h->vc[k].d_tickets;
    c.vc_partial[k] = h->vc[k].d_partial;
  }
  c.sell_tickets = h->sell.d_tickets;
  c.sell_partial = h->sell.d_partial;
  c.wc_ypart = h->wc.d_ypart;
  c.vf_tickets = h->vf.d_tickets;
  c.vf_partial = h->vf.d_partial;
}

// The combine scratch of stream s for a launch of `kernel` (vc layout k):
// *out points at a set whose buffers for that kernel exist.  A capturing
// stream takes its own set when it has one with those buffers (a warm-up
// launch on it made them), else set 0 -- nothing is allocated or
// synchronised inside a capture; the caller orders a graph's replays against
// other launches of the handle (include/hipspmv.h).
static int scratch_for(hipspmv_t* h, hipStream_t s, bool capturing, int kernel, int k,
                       hipspmv_handle::Scratch** out) {
  scratch_set0(h);  // (layouts built since the last launch)
  const uintptr_t sid = (uintptr_t)s;
  auto has = [&](const hipspmv_handle::Scratch& c) {
    if (kernel == HIPSPMV_KERNEL_SELL) return c.sell_tickets && c.sell_partial;
    if (kernel == HIPSPMV_KERNEL_WCSR) return c.wc_ypart != nullptr;
    if (kernel == HIPSPMV_KERNEL_VCACHE_FLOW) return c.vf_tickets && c.vf_partial;
    return c.vc_tickets[k] && c.vc_partial[k];
  };
  constexpr int NS = hipspmv_handle::kScratchSets;
  int si = -1;
  for (int i = 0; i < NS; ++i)
    if (h->scratch[i].assigned && h->scratch[i].sid == sid) si = i;
  if (capturing) {
    if (si < 0 || !has(h->scratch[si])) si = 0;
    if (!h->scratch[si].assigned) {
      h->scratch[si].assigned = true;
      h->scratch[si].sid = sid;
    }
  } else if (si < 0) {
    for (int i = 0; i < NS && si < 0; ++i)
      if (!h->scratch[i].assigned) si = i;
    if (si < 0) {  // a fifth stream: the least recently used set, once its launches have finished
      si = 0;
      for (int i = 1; i < NS; ++i)
        if (h->scratch[i].last < h->scratch[si].last) si = i;
      HIP_TRY(hipDeviceSynchronize());
      ++h->scratch_evictions;
    }
    h->scratch[si].assigned = true;
    h->scratch[si].sid = sid;
  }
  auto& c = h->scratch[si];
  c.last = ++h->scratch_tick;
  if (!capturing && si > 0 && !has(c)) {  // this stream's own buffers for the kernel, zeroed on it
    auto alloc = [&](auto** p, uint64_t bytes, bool zero) -> int {
      if (*p) return HIPSPMV_OK;
      bytes = std::max<uint64_t>(bytes, 8);
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), bytes));
      h->device_bytes += bytes;
      if (zero) HIP_TRY(hipMemsetAsync(*p, 0, bytes, s));
      return HIPSPMV_OK;
    };
    int st;
    if (kernel == HIPSPMV_KERNEL_SELL) {
      if ((st = alloc(&c.sell_tickets, 4ull * h->sell.ntickets, true))) return st;
      if ((st = alloc(&c.sell_partial, 8ull * h->sell.npieces, true))) return st;
    } else if (kernel == HIPSPMV_KERNEL_WCSR) {
      if ((st = alloc(&c.wc_ypart, 8ull * h->wc.nseg, false))) return st;
    } else if (kernel == HIPSPMV_KERNEL_VCACHE_FLOW) {
      if ((st = alloc(&c.vf_tickets, 4ull * h->vf.ticket_words, true))) return st;
      if ((st = alloc(&c.vf_partial, h->vf.partial_bytes, false))) return st;
    } else {
      if ((st = alloc(&c.vc_tickets[k], 4ull * h->vc[k].ticket_words, true))) return st;
      if ((st = alloc(&c.vc_partial[k], h->vc[k].partial_bytes, false))) return st;
    }
  }
  *out = &c;
  return HIPSPMV_OK;
}

static int launch(hipspmv_t* h, int kernel, const void* d_x, const void* d_y_in, void* d_y_out, int beta,
                  hipStream_t s, int mode) {
  hipError_t e = hipSuccess;
  if (mode == HIPSPMV_MODE_AUTO) mode = h->mode_opt;
  const bool scratch = kernel == HIPSPMV_KERNEL_VCACHE_SPLIT || kernel == HIPSPMV_KERNEL_VCACHE_SPLIT4 ||
                       kernel == HIPSPMV_KERNEL_WGATHER_SPLIT ||
                       kernel == HIPSPMV_KERNEL_WCSR || kernel == HIPSPMV_KERNEL_VCACHE_FLOW ||
                       (kernel == HIPSPMV_KERNEL_SELL && h->sell.npieces &&
                        (mode != HIPSPMV_MODE_ORDERED || h->dtype == HIPSPMV_U64));
  // the stream's own combine scratch: nothing is recorded or waited on between
  // launches (on one stream they are ordered by it, across streams they share
  // nothing) -- back-to-back eager launches have no packet between them
  hipspmv_handle::Scratch* sc = nullptr;
  if (scratch) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(s, &cap));
    const int k = kernel == HIPSPMV_KERNEL_VCACHE_SPLIT ? 1 : kernel == HIPSPMV_KERNEL_WGATHER_SPLIT ? 4 : 2;
    if (int st = scratch_for(h, s, cap != hipStreamCaptureStatusNone, kernel, k, &sc)) return st;
  }
  if (kernel == HIPSPMV_KERNEL_SELL) {
    const auto& q = h->sell;
    SellArgs a{q.d_off,     q.d_width,   q.d_row,     q.d_len, q.d_col,  q.d_vals,
               q.d_hubs,    h->d_rowptr, h->d_colind, h->d_vals, d_x,    d_y_in,
               d_y_out,     q.nslices,   q.nhubs,     beta,    mode == HIPSPMV_MODE_ORDERED ? 1 : 0,
               q.d_pieces,  q.npieces,   sc ? sc->sell_partial : q.d_partial, sc ? sc->sell_tickets : q.d_tickets};
    a.nt_from = h->sell_nt >= 0 ? (uint32_t)std::min<int64_t>(h->sell_nt, UINT32_MAX) : q.nslices / 2;
    h->resident_entry_bytes = q.off.empty() ? 0 : 12ull * q.off[std::min(a.nt_from, q.nslices)];
    a.chain_g = h->sell_chain_g;
    a.niso = q.niso;
    if (h->sell_only == 1) a.nslices = 0;  // experimental timing probe: the hub work alone
    if (h->sell_only == 2) a.nhubs = a.npieces = 0;  // ... or the slices alone (y incomplete)
    if (h->sell_only == 3)
      a.nslices = 0, a.nhubs = std::min(a.nhubs, 1u), a.npieces = std::min(a.npieces, 1u),
      a.niso = std::min(a.niso, 1u);
    if (h->sell_only == 2) a.niso = 0;
    e = launch_sell(h->dtype, a, s);
  } else if (kernel == HIPSPMV_KERNEL_VCACHE || kernel == HIPSPMV_KERNEL_VCACHE_SPLIT ||
      kernel == HIPSPMV_KERNEL_VCACHE_SPLIT4) {
    const int k = kernel == HIPSPMV_KERNEL_VCACHE ? 0 : kernel == HIPSPMV_KERNEL_VCACHE_SPLIT ? 1 : 2;
    const auto& v = h->vc[k];
    const VcGeom geoms[3] = {kVcOrdered, kVcSplit, v.vc4 ? kVcSplit4 : kVcQuad};
    VcacheArgs a{v.d_seg,     v.d_code,  v.d_vals,   d_x,           d_y_in,  d_y_out,
                 sc ? sc->vc_partial[k] : v.d_partial,
                 sc ? sc->vc_tickets[k] : v.d_tickets,
                 h->rows,   h->cols,    v.rows_per_block, v.nblocks, v.npanels, v.part_panels,
                 v.npad,      h->nnz - 1, v.split,   beta, h->vcache_dma, (uint32_t)geoms[k].panel,
                 h->vcache_xlane, v.max_seg, h->vcache_map};
    a.nt_from = h->vcache_nt >= 0 ? (uint32_t)std::min<int64_t>(h->vcache_nt, UINT32_MAX)
                : k < 2 || v.vc4 ? resident_blocks(v.nblocks, h->nnz) : ~0u;
    h->resident_entry_bytes = v.block_first.empty() ? 0 : 12ull * v.block_first[std::min(a.nt_from, v.nblocks)];
    a.row_runs = v.row_runs;
    if (h->vcache_xmask) a.xmask = v.d_xmask;
    // an unprofiled launch leaves an unread profile of an earlier launch readable
    // (it writes no stamps); d_prof is allocated when the option is set, never
    // here, so a profiled launch is legal only outside a capture (checked below)
    if (h->profile && k < 2) {  // the default configuration with its profile stamps
      hipStreamCaptureStatus pc = hipStreamCaptureStatusNone;
      HIP_TRY(hipStreamIsCapturing(s, &pc));
      if (pc != hipStreamCaptureStatusNone) {
        set_last_error("option profile: profiled launches cannot be captured into a graph");
        return HIPSPMV_ERR_UNSUPPORTED;
      }
      if (k == 0 && !h->d_prof) {
        set_last_error("option profile: no stamp buffer for the ordered geometry");
        return HIPSPMV_ERR_UNSUPPORTED;
      }
      if (k == 0) a.partial = h->d_prof;
      e = launch_vcache_profiled(h->dtype, a, s);
      h->prof_tickets = a.tickets;
      h->prof_pending = e == hipSuccess;
      h->prof_valid = false;
      h->prof_stream = s;
      h->prof_layout = k;
    } else if (k == 2 && v.vc4) {  // k_vcache's four-part geometry (probe)
      e = launch_vcache(h->dtype, a, s);
    } else if (k == 2) {
      a.status = h->d_status;
      a.variant = h->vquad_variant;
      e = launch_vquad(h->dtype, a, s);
    } else {
      e = launch_vcache(h->dtype, a, s);
    }
  } else if (kernel == HIPSPMV_KERNEL_VCACHE_FLOW) {
    const auto& f = h->vf;
    VflowArgs a{f.d_wbeg,  f.d_wend, f.d_code,   f.d_vals,        d_x,       d_y_in,    d_y_out,
                sc->vf_partial, sc->vf_tickets, f.d_status, h->rows, h->cols, f.rows_per_block, f.nblocks,
                f.npanels, f.part_panels, f.npad, beta};
    a.nt_from = h->vcache_nt >= 0 ? (uint32_t)std::min<int64_t>(h->vcache_nt, UINT32_MAX)
                                  : resident_blocks(f.nblocks, h->nnz);
    a.map = h->vflow_map;
    a.de = h->vflow_de;
    a.prof = h->d_vfprof;
    h->resident_entry_bytes = 12ull * f.block_first[std::min(a.nt_from, f.nblocks)];
    e = launch_vflow(h->dtype, a, s);
  } else if (kernel == HIPSPMV_KERNEL_WGATHER || kernel == HIPSPMV_KERNEL_WGATHER_SPLIT) {
    const int k = kernel == HIPSPMV_KERNEL_WGATHER ? 3 : 4;
    const auto& v = h->vc[k];
    VcacheArgs a{v.d_seg,     v.d_code,  v.d_vals,   d_x,           d_y_in,  d_y_out,
                 sc ? sc->vc_partial[k] : nullptr,
                 sc ? sc->vc_tickets[k] : nullptr,
                 h->rows,   h->cols,    v.rows_per_block, v.nblocks, v.npanels, v.part_panels,
                 v.npad,      h->nnz - 1, v.split,   beta, 0,       (uint32_t)kWgWindow.panel,
                 h->vcache_xlane, v.max_seg};
    a.chunk = h->wgather_chunk;
    if (k == 3) {
      // entries non-temporal unless option vcache_nt > 0 (full C4: 3391 us against 3594)
      a.nt_from = h->vcache_nt > 0 ? ~0u : 0u;
      h->resident_entry_bytes = a.nt_from ? 12ull * h->nnz : 0;
    } else {
      // wgather_split: row blocks b < nt_from keep their entries resident (option vcache_nt: the first
      // non-temporal block; default: the leading blocks that fit what x and y leave of
      // kWgSplitMallBytes)
      const uint64_t xy = 8ull * h->cols + 8ull * h->rows;
      const uint64_t budget = kWgSplitMallBytes > xy ? (kWgSplitMallBytes - xy) / 12 : 0;  // entries
      const uint32_t fit = (uint32_t)(std::upper_bound(v.block_first.begin(), v.block_first.end(), budget) -
                                      v.block_first.begin()) - 1;  // block_first[fit] <= budget
      a.nt_from = (uint32_t)std::min<int64_t>(h->vcache_nt >= 0 ? h->vcache_nt : fit, v.nblocks);
      a.map = h->wgather_map;
      h->resident_entry_bytes = 12ull * v.block_first[a.nt_from];
    }
    e = launch_wgather(h->dtype, a, s);
  } else if (kernel == HIPSPMV_KERNEL_WCSR) {
    const auto& w = h->wc;
    WcsrArgs a{w.d_rowptr, w.d_colind, w.d_vals, w.d_groups, w.ngroups, w.d_rowseg, w.d_segidx,
               w.d_rgroups, w.rgroups,   sc ? sc->wc_ypart : w.d_ypart, d_x, d_y_in, d_y_out, h->rows, beta};
    a.chunks = w.d_chunks;
    a.nchunks = w.nchunks;
    a.hot = w.d_hot;
    a.hotk = w.hotk;
    a.res_groups = (uint32_t)std::min<int64_t>(h->wcsr_res, w.ngroups);
    h->resident_entry_bytes = w.group_first.empty() ? 0 : 12ull * w.group_first[a.res_groups];
    a.cols = h->cols;
    a.xcd = h->wcsr_xcd;
    if (h->wcsr_reduce == 0 && w.d_rrow) {  // the compact reduce (default; option wcsr_reduce 1: all rows)
      a.rrow = w.d_rrow;
      a.rsegc = w.d_rsegc;
      a.nebits = w.d_nebits;
      a.cgroups = w.d_cgroups;
      a.ncgroups = w.ncgroups;
      a.fill_early = h->wcsr_fill >= 0 ? h->wcsr_fill : 3ull * (h->rows - w.nrows_ne) >= 2ull * h->rows;
    }
    e = launch_wcsr(h->dtype, a, s);
  } else {
    CsrArgs a{h->d_rowptr, h->d_colind, h->d_vals, d_x, d_y_in, d_y_out, h->d_groups, h->rows, h->ngroups, beta};
    h->resident_entry_bytes = 12ull * h->nnz;  // (default policy throughout)
    e = kernel == HIPSPMV_KERNEL_CSR_LANE ? launch_csr_lane(h->dtype, a, s) : launch_csr_vector(h->dtype, a, s);
  }
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  h->last_kernel = kernel;
  h->last_beta = beta;
  h->execs++;
  return HIPSPMV_OK;
}

// k_vquad's combine fallbacks: owners that gave up waiting for their share's
// publishers and published their own share too (csrc/combine.h) since create.
// The result is exact on either path; the count says which one ran (variant 20
// forces it).  Read by the stat key "handoff_fallbacks" only, never per exec.
static int read_status(hipspmv_t* h, uint32_t* out) {
  *out = 0;
  if (!h->d_status) return HIPSPMV_OK;
  DeviceGuard g(h->device);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, h->d_status, 4, hipMemcpyDeviceToHost));
  return HIPSPMV_OK;
}

// The last kernel's symbol prefix in a rocprofv3 CSV (dtype-qualified where
// one kernel template has several geometries)
static std::string kernel_symbol(const hipspmv_t* h) {
  const std::string T = h->dtype == HIPSPMV_U64 ? "unsigned long" : "double";
  switch (h->last_kernel) {
    case HIPSPMV_KERNEL_VCACHE: return "k_vcache<" + T + ", 1,";
    case HIPSPMV_KERNEL_VCACHE_SPLIT: return "k_vcache<" + T + ", 3,";
    case HIPSPMV_KERNEL_VCACHE_SPLIT4: return "k_vquad<" + T + ",";
    case HIPSPMV_KERNEL_WGATHER: return "k_wgather<" + T + ",";
    case HIPSPMV_KERNEL_WGATHER_SPLIT: return "k_wgather_split<" + T + ",";
    case HIPSPMV_KERNEL_CSR_LANE: return "k_csr_lane<" + T + ">";
    case HIPSPMV_KERNEL_CSR_VECTOR: return "k_csr_vector<" + T + ", false>";
    case HIPSPMV_KERNEL_WCSR: return "k_csr_vector<" + T + ", true>";
    case HIPSPMV_KERNEL_VCACHE_FLOW: return "k_vflow<" + T + ",";
    case HIPSPMV_KERNEL_SELL: return "k_sell";
    default: return "hipspmv::";
  }
}

// A counter of the attached PMC CSV for the last kernel: true and *v set when
// the CSV holds it
static bool pmc_value(const hipspmv_t* h, const char* counter, uint64_t* v) {
  if (h->pmc_csv.empty()) return false;
  double m = 0;
  uint64_t n = 0;
  if (hipspmv_pmc_counter(h->pmc_csv.c_str(), kernel_symbol(h).c_str(), counter, &m, &n) != HIPSPMV_OK || !n)
    return false;
  *v = (uint64_t)std::llround(m);
  return true;
}

static int resolve_pending(hipspmv_t* h) {
  if (!h->pending) return HIPSPMV_OK;
  DeviceGuard g(h->device);
  HIP_TRY(hipEventSynchronize(h->ev[2]));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, h->ev[1], h->ev[2]));
  h->kernel_ns = (uint64_t)(ms * 1e6);
  h->pending = false;
  return HIPSPMV_OK;
}

// The NewCache state statistics of the last profiled launch, from its stamps
// (csrc/vcache.hip, AB bit 128): means over the workgroups, converted to
// shader cycles at the handle's clock (s_memrealtime ticks are 10 ns).
static int resolve_profile(hipspmv_t* h) {
  if (!h->prof_pending) return HIPSPMV_OK;
  DeviceGuard g(h->device);
  HIP_TRY(hipStreamSynchronize(h->prof_stream));
  const auto& v = h->vc[h->prof_layout];
  const uint32_t units = v.nblocks * v.split;
  std::vector<uint32_t> st((size_t)kVcProfWords * units);
  const uint32_t* src = h->prof_layout == 0 ? h->d_prof : h->prof_tickets + 4ull * v.nblocks;
  HIP_TRY(hipMemcpy(st.data(), src, 4ull * st.size(), hipMemcpyDeviceToHost));
  const double cyc_per_tick = h->clock_khz / 1e5;
  auto at = [&](uint32_t u, int k) { return st[(size_t)kVcProfWords * u + k]; };
  uint32_t t_end = at(0, 3);
  for (uint32_t u = 1; u < units; ++u)
    if ((int32_t)(at(u, 3) - t_end) > 0) t_end = at(u, 3);
  uint32_t t_beg = at(0, 0);
  for (uint32_t u = 1; u < units; ++u)
    if ((int32_t)(at(u, 0) - t_beg) < 0) t_beg = at(u, 0);
  double fill = 0, active = 0, flush = 0, done = 0, lw = 0, lwait = 0, cwait = 0;
  for (uint32_t u = 0; u < units; ++u) {
    fill += (uint32_t)(at(u, 1) - at(u, 0));
    active += (uint32_t)(at(u, 2) - at(u, 1));
    flush += (uint32_t)(at(u, 3) - at(u, 2));
    done += (uint32_t)(t_end - at(u, 3));
    lw += at(u, 5);
    lwait += at(u, 6);
    cwait += at(u, 7);
  }
  auto mean_cyc = [&](double ticks) { return (uint64_t)std::llround(ticks / units * cyc_per_tick); };
  auto mean = [&](double c) { return (uint64_t)std::llround(c / units); };
  h->prof = hipspmv_handle::Prof{mean_cyc(fill), mean_cyc(active), mean_cyc(flush), mean_cyc(done), mean(lw),
                                 mean(lwait), mean(cwait), units,
                                 (uint64_t)std::llround((uint32_t)(t_end - t_beg) * cyc_per_tick)};
  h->prof_pending = false;
  h->prof_valid = true;
  return HIPSPMV_OK;
}

extern "C" {

int hipspmv_create(const uint32_t* colptr, const uint32_t* rowind, const void* vals, uint32_t rows, uint32_t cols,
                   uint32_t nnz, int dtype, int device, hipspmv_t** out) {
  if (!colptr || (nnz && (!rowind || !vals))) return HIPSPMV_ERR_INVALID_ARG;
  try {
    return create_common(rows, cols, nnz, dtype, device, out, [&](HostCSR& a, std::string& why) {
      return csc_to_csr(colptr, rowind, vals, rows, cols, nnz, a, why);
    });
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    return HIPSPMV_ERR_INVALID_ARG;
  }
}

int hipspmv_create_csr(const uint32_t* rowptr, const uint32_t* colind, const void* vals, uint32_t rows,
                       uint32_t cols, uint32_t nnz, int dtype, int device, hipspmv_t** out) {
  if (!rowptr || (nnz && (!colind || !vals))) return HIPSPMV_ERR_INVALID_ARG;
  try {
    return create_common(rows, cols, nnz, dtype, device, out, [&](HostCSR& a, std::string& why) {
      return copy_csr(rowptr, colind, vals, rows, cols, nnz, a, why);
    });
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    return HIPSPMV_ERR_INVALID_ARG;
  }
}

int hipspmv_set_option(hipspmv_t* h, const char* key, int64_t value) {
  if (!h || !key) return HIPSPMV_ERR_INVALID_ARG;
  const std::string k(key);
  if (k == "kernel") {
    if (value < HIPSPMV_KERNEL_AUTO || value > HIPSPMV_KERNEL_WGATHER_SPLIT) return HIPSPMV_ERR_INVALID_ARG;
    if ((value == HIPSPMV_KERNEL_VCACHE_SPLIT4 || value == HIPSPMV_KERNEL_VCACHE_FLOW) && !kExperimental)
      return HIPSPMV_ERR_UNSUPPORTED;
    if (value == HIPSPMV_KERNEL_VCACHE && !h->vc0_eligible) return HIPSPMV_ERR_UNSUPPORTED;
    if (value == HIPSPMV_KERNEL_WGATHER && !h->wg_eligible) return HIPSPMV_ERR_UNSUPPORTED;
    if (value == HIPSPMV_KERNEL_WGATHER_SPLIT && !h->wgs_eligible) return HIPSPMV_ERR_UNSUPPORTED;
    if (int st = ensure_layout(h, (int)value)) return st;
    h->kernel_opt = (int)value;
  } else if (k == "vcache_dma") {
    if (value < -1 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    if (value == 1 && !kExperimental) return HIPSPMV_ERR_UNSUPPORTED;  // (the split geometry's loaders are DMA)
    h->vcache_dma = (int)value;
  } else if (k == "vcache_map") {  // 1: split4 XCD pairs; 2: split, one column part per XCD where it can
    if (value < 0 || value > 2) return HIPSPMV_ERR_INVALID_ARG;
    if (value && !kExperimental) return HIPSPMV_ERR_UNSUPPORTED;
    h->vcache_map = (int)value;
  } else if (k == "vflow_map") {  // 1: k_vflow's column part h on XCDs 2h and 2h + 1
    if (value < 0 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->vflow_map = (int)value;
  } else if (k == "vflow_prof") {  // diagnostic: k_vflow launches write per-wave cycle stamps
    DeviceGuard g(h->device);
    if (value && !h->d_vfprof) {
      const size_t bytes = 4ull * 4 * 16 * 4096;  // 4 words x 16 waves x up to 4096 units
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&h->d_vfprof), bytes));
      HIP_TRY(hipMemset(h->d_vfprof, 0, bytes));
      h->device_bytes += bytes;
    } else if (!value && h->d_vfprof) {
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipFree(h->d_vfprof));
      h->d_vfprof = nullptr;
    }
  } else if (k == "vflow_de") {  // k_vflow's entry ring depth
    if (value != 2 && value != 3 && value != 4 && value != 8) return HIPSPMV_ERR_INVALID_ARG;
    h->vflow_de = (int)value;
  } else if (k == "vcache_xmask") {
    if (value < 0 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->vcache_xmask = (int)value;
  } else if (k == "vquad_variant") {  // k_vquad configuration (csrc/vquad.hip)
    if (value < 0 || value > 26) return HIPSPMV_ERR_INVALID_ARG;
    if (!kExperimental) return HIPSPMV_ERR_UNSUPPORTED;
    // 6-16 are timing ablations that give wrong y (or race): experimental builds only
    const char* exp = std::getenv("HIPSPMV_EXPERIMENTAL");
    if (value >= 6 && value <= 16 && !(exp && std::strcmp(exp, "1") == 0)) return HIPSPMV_ERR_UNSUPPORTED;
    if (h->vc[2].ok && h->vc[2].max_seg > vquad_max_window((int)value)) return HIPSPMV_ERR_UNSUPPORTED;
    h->vquad_variant = (int)value;
  } else if (k == "wgather_chunk") {  // row blocks per k_wgather launch (0: all in one launch)
    if (value < 0 || value > (int64_t)UINT32_MAX) return HIPSPMV_ERR_INVALID_ARG;
    h->wgather_chunk = (uint32_t)value;
  } else if (k == "sell_only") {  // experimental timing probe: 1 hub work only, 2 slices only (y incomplete)
    const char* exp = std::getenv("HIPSPMV_EXPERIMENTAL");
    if (value < 0 || value > 3) return HIPSPMV_ERR_INVALID_ARG;  // 3: the first (longest) hub row alone
    if (value && !(exp && std::strcmp(exp, "1") == 0)) return HIPSPMV_ERR_UNSUPPORTED;
    h->sell_only = (int)value;
  } else if (k == "sell_chain") {  // experimental ORDERED hub chains: 1 none isolated, 2 / 3: G = 12 / 30
    if (value < 0 || value > 3) return HIPSPMV_ERR_INVALID_ARG;
    const char* exp = std::getenv("HIPSPMV_EXPERIMENTAL");
    if (value && !(exp && std::strcmp(exp, "1") == 0)) return HIPSPMV_ERR_UNSUPPORTED;
    h->sell_chain_g = (uint32_t)value;
  } else if (k == "sell_nt") {  // first SELL slice whose entries load non-temporally (-1: half)
    if (value < -1 || value > (int64_t)UINT32_MAX) return HIPSPMV_ERR_INVALID_ARG;
    h->sell_nt = value;
  } else if (k == "wcsr_fill") {  // 1: empty rows filled beside the segment pass; 0: after the reduce; -1: by rule
    if (value < -1 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->wcsr_fill = (int)value;
  } else if (k == "wgather_map") {  // wgather_split: 0 halves by XCD (default), 1 alternating (A/B); same bits
    if (value < 0 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->wgather_map = (int)value;
  } else if (k == "wcsr_xcd") {  // 1: segment-pass blocks by XCD eighths of the window order; same bits
    if (value < 0 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->wcsr_xcd = (int)value;
  } else if (k == "wcsr_reduce") {  // 0: compact reduce over the rows with segments (default); 1: every row
    if (value < 0 || value > 1) return HIPSPMV_ERR_INVALID_ARG;
    h->wcsr_reduce = (int)value;
  } else if (k == "wcsr_res") {  // wcsr segment-pass groups below it keep their entries resident
    if (value < 0 || value > (int64_t)UINT32_MAX) return HIPSPMV_ERR_INVALID_ARG;
    h->wcsr_res = value;
  } else if (k == "vcache_nt") {  // first row block whose entries load non-temporally (-1: per geometry)
    if (value < -1 || value > (int64_t)UINT32_MAX) return HIPSPMV_ERR_INVALID_ARG;
    h->vcache_nt = value;
  } else if (k == "vcache_xlane") {
    if (value < -1 || value > 6) return HIPSPMV_ERR_INVALID_ARG;
    // the product build has the split geometry's 0 / 3 / 5 (and the ordered geometry's 0, which 6 shares)
    if ((value == 1 || value == 2 || value == 4) && !kExperimental) return HIPSPMV_ERR_UNSUPPORTED;
    h->vcache_xlane = (int)value;
  } else if (k == "mode") {
    if (value != HIPSPMV_MODE_ORDERED && value != HIPSPMV_MODE_FAST) return HIPSPMV_ERR_INVALID_ARG;
    h->mode_opt = (int)value;
  } else if (k == "timing") {
    h->timing = value ? 1 : 0;
  } else if (k == "profile") {  // NewCache state statistics from the vcache kernels' stamps
    if (value && h->vc0_eligible && !h->d_prof) {  // the ordered geometry's stamp buffer, allocated here
      DeviceGuard g(h->device);
      const size_t b = 4ull * kVcProfWords * h->vc[0].nblocks;
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&h->d_prof), b));
      h->device_bytes += b;
    }
    h->profile = value ? 1 : 0;
  } else {
    return HIPSPMV_ERR_KEY;
  }
  return HIPSPMV_OK;
}

int hipspmv_exec(hipspmv_t* h, const void* x, void* y, int beta, int mode) {
  if (!h || !x || !y || (beta != 0 && beta != 1)) return HIPSPMV_ERR_INVALID_ARG;
  const int kernel = choose_kernel(h, mode);
  if (kernel < 0) return -kernel;
  if (int st = ensure_layout(h, kernel)) return st;
  try {
    DeviceGuard g(h->device);
    const size_t bx = 8ull * h->cols, by = 8ull * h->rows;
    if (!h->d_x) {
      HIP_TRY(hipMalloc(&h->d_x, bx));
      h->device_bytes += bx;
    }
    if (!h->d_y) {
      HIP_TRY(hipMalloc(&h->d_y, by));
      h->device_bytes += by;
    }
    hipStream_t s = h->stream;  // (its own combine scratch set: no ordering against other streams)
    HIP_TRY(hipEventRecord(h->ev[0], s));
    HIP_TRY(hipMemcpyAsync(h->d_x, x, bx, hipMemcpyHostToDevice, s));
    if (beta) HIP_TRY(hipMemcpyAsync(h->d_y, y, by, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(h->ev[1], s));
    int st = launch(h, kernel, h->d_x, h->d_y, h->d_y, beta, s, mode);
    if (st) return st;
    HIP_TRY(hipEventRecord(h->ev[2], s));
    HIP_TRY(hipMemcpyAsync(y, h->d_y, by, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(h->ev[3], s));
    HIP_TRY(hipStreamSynchronize(s));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    h->h2d_ns = (uint64_t)(ms * 1e6);
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[1], h->ev[2]));
    h->kernel_ns = (uint64_t)(ms * 1e6);
    HIP_TRY(hipEventElapsedTime(&ms, h->ev[2], h->ev[3]));
    h->d2h_ns = (uint64_t)(ms * 1e6);
    h->pending = false;
    return HIPSPMV_OK;
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    set_last_error("unexpected C++ exception");
    return HIPSPMV_ERR_HIP;
  }
}

int hipspmv_exec_device(hipspmv_t* h, const void* d_x, const void* d_y_in, void* d_y_out, int beta, int mode,
                        void* stream) {
  if (!h || !d_x || !d_y_out || (beta != 0 && beta != 1) || (beta && !d_y_in)) return HIPSPMV_ERR_INVALID_ARG;
  const int kernel = choose_kernel(h, mode);
  if (kernel < 0) return -kernel;
  if (int st = ensure_layout(h, kernel)) return st;
  DeviceGuard g(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);  // NULL: the default stream
  if (h->timing) HIP_TRY(hipEventRecord(h->ev[1], s));
  int st = launch(h, kernel, d_x, beta ? d_y_in : d_y_out, d_y_out, beta, s, mode);
  if (st) return st;
  if (h->timing) {
    HIP_TRY(hipEventRecord(h->ev[2], s));
    h->pending = true;
  }
  return HIPSPMV_OK;
}

int hipspmv_stat(hipspmv_t* h, const char* key, uint64_t* out) {
  if (!h || !key || !out) return HIPSPMV_ERR_INVALID_ARG;
  const std::string k(key);
  const uint64_t alg = 12ull * h->nnz + 4ull * (h->rows + 1ull) + 8ull * h->cols + 8ull * h->rows;
  if (k == "rows") *out = h->rows;
  else if (k == "cols") *out = h->cols;
  else if (k == "nz") *out = h->nnz;
  else if (k == "dtype") *out = (uint64_t)h->dtype;
  else if (k == "device") *out = (uint64_t)h->device;
  else if (k == "kernel") *out = (uint64_t)h->last_kernel;
  else if (k == "setup_ns") *out = h->setup_ns + h->layout_ns;
  else if (k == "create_ns") *out = h->setup_ns;
  else if (k == "layout_ns") *out = h->layout_ns;
  else if (k == "setup_csr_ns") *out = h->setup_csr_ns;
  else if (k == "setup_upload_ns") *out = h->setup_upload_ns;
  else if (k == "setup_scan_ns") *out = h->setup_scan_ns;
  else if (k == "setup_layouts_ns") *out = h->setup_layouts_ns;
  else if (k == "auto_fallback") *out = (uint64_t)h->auto_fallback;
  else if (k == "wgather_chunk") *out = h->wgather_chunk;
  else if (k == "kernel_ns") {
    int st = resolve_pending(h);
    if (st) return st;
    *out = h->kernel_ns;
  } else if (k == "h2d_ns") *out = h->h2d_ns;
  else if (k == "d2h_ns") *out = h->d2h_ns;
  else if (k == "alg_bytes") *out = alg;
  else if (k == "alg_bytes_beta1") *out = alg + 8ull * h->rows;
  else if (k == "flops") *out = 2ull * h->nnz;
  else if (k == "device_bytes") *out = h->device_bytes;
  else if (k == "vcache_blocks") *out = h->vc[0].nblocks;
  else if (k == "vcache_panels") *out = h->vc[0].npanels;
  else if (k == "vcache_rows_per_block") *out = h->vc[0].rows_per_block;
  else if (k == "vcache_max_segment") *out = h->vc[0].max_seg;
  else if (k == "vcache_eligible") *out = h->vc0_eligible;
  else if (k == "vcache_split_eligible") *out = h->vc[1].ok;
  else if (k == "vcache_split_units") *out = (uint64_t)h->vc[1].nblocks * h->vc[1].split;
  else if (k == "vcache_split_rows_per_block") *out = h->vc[1].rows_per_block;
  // x bytes a launch streams from L2/MALL into LDS: every row block reads all
  // columns once (split: its two halves read one half each)
  else if (k == "vcache_x_bytes") *out = h->vc0_eligible ? 8ull * h->vc[0].nblocks * h->cols : 0;
  else if (k == "vcache_split_x_bytes") *out = h->vc[1].ok ? 8ull * h->vc[1].nblocks * h->cols : 0;
  // the four-part geometry's eligibility by shape (a read builds nothing, ADVICE r05: selecting
  // the kernel builds the layout, which can still prove unplaceable -- HIPSPMV_ERR_UNSUPPORTED)
  else if (k == "vcache_split4_eligible") *out = h->vc[2].ok || h->vq_eligible;
  else if (k == "scratch_evictions") *out = h->scratch_evictions;
  else if (k == "vflow_eligible") *out = h->vf.ok;
  else if (k.rfind("vflow_prof_", 0) == 0) {  // means over the units of the last profiled launch, cycles
    // vflow_prof_loader_{freewait,dma,total}, vflow_prof_compute_{panelwait,apply,loads,total}
    if (!h->d_vfprof || !h->vf.ok) return HIPSPMV_ERR_UNSUPPORTED;
    DeviceGuard g(h->device);
    const uint32_t units = h->vf.nblocks * kVfGeom.split;
    std::vector<uint32_t> st(4ull * 16 * units);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(st.data(), h->d_vfprof, 4 * st.size(), hipMemcpyDeviceToHost));
    const std::string f = k.substr(11);
    const bool loader = f.rfind("loader_", 0) == 0;
    const std::string what = f.substr(loader ? 7 : 8);
    const int idx = loader ? (what == "freewait" ? 0 : what == "dma" ? 1 : what == "total" ? 3 : -1)
                           : (what == "panelwait" ? 0 : what == "apply" ? 1 : what == "loads" ? 2 : what == "total" ? 3 : -1);
    if (idx < 0) return HIPSPMV_ERR_KEY;
    double sum = 0;
    uint64_t n = 0;
    for (uint32_t u = 0; u < units; ++u)
      for (int w = loader ? 0 : kVfLoaders; w < (loader ? kVfLoaders : 16); ++w, ++n) sum += st[4ull * (u * 16 + w) + idx];
    *out = n ? (uint64_t)(sum / n) : 0;
  }  // the k_vflow layout is built (selected, and it fits)
  else if (k == "vflow_units") *out = (uint64_t)h->vf.nblocks * kVfGeom.split;
  else if (k == "vflow_max_group") *out = h->vf.max_group;
  else if (k == "vflow_x_bytes") *out = h->vf.ok ? 8ull * h->vf.nblocks * h->cols : 0;
  else if (k == "vflow_timeouts") {  // a k_vflow flag wait gave up since the layout was built (results wrong)
    uint32_t v = 0;
    if (h->vf.d_status) {
      DeviceGuard g(h->device);
      HIP_TRY(hipDeviceSynchronize());
      HIP_TRY(hipMemcpy(&v, h->vf.d_status, 4, hipMemcpyDeviceToHost));
    }
    *out = (v >> 1) & 1u;
  }
  // entry bytes the last launch loaded with the default cache policy -- they may stay in the 256 MiB
  // Infinity Cache until the next launch (options vcache_nt / sell_nt / wcsr_res); the rest non-temporal
  else if (k == "resident_entry_bytes") *out = h->resident_entry_bytes;  // a fifth stream took over a scratch set
  else if (k == "scratch_streams") {  // streams holding a combine scratch set
    *out = 0;
    for (const auto& c : h->scratch) *out += c.assigned;
  }
  else if (k == "wgather_eligible") *out = h->vc[3].ok || h->wg_eligible;
  else if (k == "wgather_max_run") *out = h->wg_max_run;
  else if (k == "vcache_max_run") *out = h->vc[0].max_run;
  else if (k == "vcache_split_max_run") *out = h->vc[1].max_run;
  else if (k == "wgather_windows") *out = h->vc[3].npanels;
  else if (k == "wgather_split_eligible") *out = h->vc[4].ok || h->wgs_eligible;
  else if (k == "wgather_split_rows_per_block") *out = h->vc[4].rows_per_block;
  else if (k == "wgather_split_units") *out = (uint64_t)h->vc[4].nblocks * kWgSplit.split;
  else if (k == "vcache_split4_x_bytes") *out = h->vc[2].ok ? 8ull * h->vc[2].nblocks * h->cols : 0;
  else if (k == "wcsr_segments") *out = h->wc.built ? h->wc.nseg : h->wc_segments;
  else if (k == "wcsr_max_segment") *out = h->wc.max_seg;
  else if (k == "wcsr_window_log2") *out = h->wc.built ? h->wc.log2w : kWcLog2Window;
  else if (k == "wcsr_chunks") *out = h->wc.nchunks;
  else if (k == "wcsr_hot") *out = h->wc.hotk;
  else if (k == "wcsr_groups") *out = h->wc.ngroups;
  else if (k == "wcsr_reduce_groups") *out = h->wc.built ? (h->wcsr_reduce == 0 ? h->wc.ncgroups : h->wc.rgroups) : 0;
  else if (k == "wcsr_rows_with_segments") *out = h->wc.nrows_ne;
  else if (k == "sell_slices") *out = h->sell.nslices;
  else if (k == "sell_hubs") *out = h->sell.nhubs;
  else if (k == "sell_iso_hubs") *out = h->sell.niso;
  else if (k == "sell_hub_pieces") *out = h->sell.npieces;
  else if (k == "sell_padding") *out = h->sell.padding;
  else if (k == "row_groups") *out = h->ngroups;
  else if (k == "max_row_len") *out = h->max_row_len;
  else if (k == "empty_rows") *out = h->empty_rows;
  else if (k == "execs") *out = h->execs;
  // k_vquad owners that gave up waiting (publish-and-count path), since create; "handoff_timeouts"
  // is its round-4 name, kept as an alias
  else if (k == "handoff_fallbacks" || k == "handoff_timeouts") {
    uint32_t v = 0;
    if (int st = read_status(h, &v)) return st;
    *out = v;
  }
  else if (k == "vquad_variant") *out = (uint64_t)h->vquad_variant;
  else if (k == "vcache_split4_max_segment") *out = h->vc[2].max_seg;
  else if (k == "clock_khz") *out = (uint64_t)h->clock_khz;
  // The reference accelerator's cache statistics (HardwareSpMVNewCache.cpp:
  // 189-204), restated for the last kernel's layout:
  else if (k == "pmc_attached") *out = h->pmc_csv.empty() ? 0 : 1;
  else if ((k == "read_misses" && pmc_value(h, "TCC_MISS", out)) ||
           (k == "hazard_stalls" && pmc_value(h, "SQ_LDS_BANK_CONFLICT", out)) ||
           (k == "capacity_stalls" && pmc_value(h, "TCP_PENDING_STALL_CYCLES", out))) {
    // measured: the attached counter CSV's mean per dispatch of the last kernel (L2 misses, LDS
    // bank-conflict cycles, L1 cycles stalled on requests pending at L2), DESIGN.md §6.9
  } else if (k == "read_misses" || k == "hazard_stalls" || k == "ocm_depth" || k == "read_misses_model" ||
             k == "hazard_stalls_model") {
    const int kn = h->last_kernel;
    const int li = kn == HIPSPMV_KERNEL_VCACHE ? 0 : kn == HIPSPMV_KERNEL_VCACHE_SPLIT ? 1
                 : kn == HIPSPMV_KERNEL_VCACHE_SPLIT4 ? 2 : kn == HIPSPMV_KERNEL_WGATHER ? 3
                 : kn == HIPSPMV_KERNEL_WGATHER_SPLIT ? 4 : -1;
    const bool lds_x = li >= 0 && li < 3;  // x panels staged in LDS (wgather gathers x from L2)
    if (k == "read_misses" || k == "read_misses_model")  // x words not held on chip when a product needs them
      *out = lds_x ? (uint64_t)h->vc[li].nblocks * h->cols : (uint64_t)h->nnz;
    else if (k == "hazard_stalls" || k == "hazard_stalls_model")  // adds waiting on the previous add to their y row
      *out = li >= 0 ? h->vc[li].n_cont
           : kn == HIPSPMV_KERNEL_CSR_VECTOR ? 0 : (uint64_t)h->nnz - (h->rows - h->empty_rows);
    else  // on-chip vector words per workgroup: the y block + the two x panels
      *out = li >= 0 ? (uint64_t)h->vc[li].rows_per_block +
                           (lds_x ? 2ull * (li == 0 ? kVcOrdered.panel : li == 1 ? kVcSplit.panel : kVcSplit4.panel) : 0)
                     : 0;
  } else if (k == "profile" || k == "profiled" || k == "profile_units" || k == "profile_span_cycles" ||
             k.rfind("state_", 0) == 0 || k == "no_valid_but_ready" || k == "no_ready_but_valid") {
    // the reference's cache-FSM state counts and stream-monitor stalls
    // (HardwareSpMVNewCache.cpp:130-204, NoWMVectorCache.scala:162-292),
    // measured by the last profiled launch
    if (int st = resolve_profile(h)) return st;
    const auto& p = h->prof;
    const bool ok = h->prof_valid;
    if (k == "profile") *out = (uint64_t)h->profile;
    else if (k == "profiled") *out = ok;
    else if (k == "profile_units") *out = ok ? p.units : 0;
    else if (k == "profile_span_cycles") *out = ok ? p.span : 0;
    else if (k == "state_fill") *out = ok ? p.fill : 0;        // y block initialised, first x panel staged
    else if (k == "state_active") *out = ok ? p.active : 0;    // the panel steps
    else if (k == "state_flush") *out = ok ? p.flush : 0;      // column-part combine and y written back
    else if (k == "state_done") *out = ok ? p.done : 0;        // finished, waiting for the launch's last workgroup
    else if (k == "state_read_miss1") *out = 0;                // no write-before-miss ordering on the GPU
    else if (k == "state_read_miss2") *out = ok ? p.loader_work : 0;  // fetching x panels (loader wave, per step)
    else if (k == "state_read_miss3") *out = 0;                // LDS-DMA lands panels without a fill step
    else if (k == "state_cold_miss") *out = h->last_beta ? 0 : h->rows;  // rows started at +0.0 without a read
    else if (k == "no_valid_but_ready") *out = ok ? p.compute_wait : 0;  // compute waves waiting on the panel
    else if (k == "no_ready_but_valid") *out = ok ? p.loader_wait : 0;   // panel ready, compute still busy
    else return HIPSPMV_ERR_KEY;
  } else if (k == "issue_window") {  // entries one workgroup keeps in flight (vcache family), else 0
    const int kn = h->last_kernel;
    *out = kn == HIPSPMV_KERNEL_VCACHE ? 4ull * 3 * 8 * 64 : kn == HIPSPMV_KERNEL_VCACHE_SPLIT ? 4ull * 2 * 13 * 64 : 0;
  } else if (k == "capacity_stalls" || k == "cms") {
    // capacity stalls: no fixed issue window (the hardware analogue is
    // TCP_PENDING_STALL_CYCLES, tools/cache_stats.py); cms: the kernels mask
    // the cold-miss-skip bits at create and never use them
    *out = 0;
  } else if (k == "total_cycles" || k == "active_cycles") {
    int st = resolve_pending(h);
    if (st) return st;
    const double ghz = h->clock_khz / 1e6;
    // total: the last launch at the shader clock; active: the cycles it would
    // take at the HBM roofline (8 TB/s) -- active/total = roofline fraction
    *out = (uint64_t)std::ceil(k == "total_cycles" ? h->kernel_ns * ghz : alg / 8000.0 * ghz);
  }
  else return HIPSPMV_ERR_KEY;
  return HIPSPMV_OK;
}

const char* hipspmv_kernel_name(hipspmv_t* h, int mode) {
  if (!h) return "invalid";
  switch (choose_kernel(h, mode)) {
    case HIPSPMV_KERNEL_VCACHE: return "vcache";
    case HIPSPMV_KERNEL_VCACHE_SPLIT: return "vcache_split";
    case HIPSPMV_KERNEL_VCACHE_SPLIT4: return "vcache_split4";
    case HIPSPMV_KERNEL_WGATHER: return "wgather";
    case HIPSPMV_KERNEL_WGATHER_SPLIT: return "wgather_split";
    case HIPSPMV_KERNEL_CSR_LANE: return "csr_lane";
    case HIPSPMV_KERNEL_CSR_VECTOR: return "csr_vector";
    case HIPSPMV_KERNEL_SELL: return "sell";
    case HIPSPMV_KERNEL_WCSR: return "wcsr";
    case HIPSPMV_KERNEL_VCACHE_FLOW: return "vcache_flow";
    default: return "unsupported";
  }
}

int hipspmv_attach_pmc(hipspmv_t* h, const char* csv_path) {
  if (!h) return HIPSPMV_ERR_INVALID_ARG;
  if (!csv_path || !*csv_path) {
    h->pmc_csv.clear();
    return HIPSPMV_OK;
  }
  std::ifstream probe(csv_path);
  if (!probe) {
    set_last_error(std::string("pmc: cannot open ") + csv_path);
    return HIPSPMV_ERR_INVALID_ARG;
  }
  h->pmc_csv = csv_path;
  return HIPSPMV_OK;
}

int hipspmv_destroy(hipspmv_t* h) {
  if (!h) return HIPSPMV_ERR_INVALID_ARG;
  release(h);
  return HIPSPMV_OK;
}

int hipspmv_release_wait(void) {
  Reclaimer::get().wait();
  return HIPSPMV_OK;
}

int hipspmv_prep_stats(const uint32_t* colptr, const uint32_t* rowind, uint32_t rows, uint32_t cols, uint32_t nnz,
                       int device, hipspmv_prep_stats_t* out) {
  try {
    return prep_stats(colptr, rowind, rows, cols, nnz, device, out);
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    set_last_error("unexpected C++ exception");
    return HIPSPMV_ERR_HIP;
  }
}

int hipspmv_mark_row_starts(const uint32_t* rowind, uint32_t* rowind_out, uint32_t rows, uint32_t nnz, int reverse,
                            int shift, int device, uint64_t* kernel_ns) {
  try {
    return mark_row_starts(rowind, rowind_out, rows, nnz, reverse, shift, device, kernel_ns);
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    set_last_error("unexpected C++ exception");
    return HIPSPMV_ERR_HIP;
  }
}

const char* hipspmv_strerror(int status) {
  switch (status) {
    case HIPSPMV_OK: return "ok";
    case HIPSPMV_ERR_INVALID_ARG: return "invalid argument";
    case HIPSPMV_ERR_INVALID_MATRIX: return "invalid matrix";
    case HIPSPMV_ERR_HIP: return "HIP runtime error";
    case HIPSPMV_ERR_OOM: return "out of memory";
    case HIPSPMV_ERR_UNSUPPORTED: return "unsupported kernel/option for this matrix";
    case HIPSPMV_ERR_NO_DEVICE: return "no such device";
    case HIPSPMV_ERR_KEY: return "unknown key";
    default: return "unknown status";
  }
}

const char* hipspmv_last_error(void) { return g_last_error.c_str(); }

int hipspmv_abi_version(void) { return HIPSPMV_ABI_VERSION; }

int hipspmv_build_flags(void) { return kExperimental ? HIPSPMV_BUILD_EXPERIMENTAL : 0; }

int hipspmv_device_count(int* count) {
  if (!count) return HIPSPMV_ERR_INVALID_ARG;
  *count = 0;
  hipError_t e = hipGetDeviceCount(count);
  if (e == hipErrorNoDevice) {
    *count = 0;
    return HIPSPMV_OK;
  }
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  return HIPSPMV_OK;
}

}  // extern "C"
