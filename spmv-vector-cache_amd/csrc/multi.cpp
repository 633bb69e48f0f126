// hipspmv_multi_*: one matrix row-partitioned over several devices of this
// process (SURVEY.md §8(b) "ndev", §8(e)), the in-process counterpart of
// bench.py's one-process-per-GPU run.  Built only on the public C ABI (one
// hipspmv_t per shard) plus the HIP runtime and RCCL.
//
//   create: CSC -> CSR once (or a CSR taken as is), rows cut into ndev
//           contiguous cost-balanced blocks starting at multiples of
//           HIPSPMV_SHARD_ALIGN rows (hipspmv_partition_rows: entries +
//           wcsr segments + rows, plan.cpp partition_rows_cost), block i
//           uploaded to devices[i].
//   exec:   x host -> devices[0]; broadcast devices[0] -> all others (RCCL
//           ncclBroadcast over xGMI, one communicator per device, from one
//           thread in an ncclGroupStart/End; with repeated device ids, where
//           RCCL refuses a communicator, peer copies instead); every shard's
//           kernel on its own stream; y slices back into their rows of y.
// There is no cross-device reduction, so every row is computed exactly as a
// single-device handle computes it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "hipspmv.h"
#include "hipspmv_internal.h"

using namespace hipspmv;

namespace {

// RCCL entry points, resolved at first use so libhipspmv.so does not depend
// on librccl at load time (it is only needed for multi-device handles).
struct Rccl {
  ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  const char* (*errorString)(ncclResult_t) = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return x;
    x.commInitAll = reinterpret_cast<decltype(x.commInitAll)>(dlsym(lib, "ncclCommInitAll"));
    x.commDestroy = reinterpret_cast<decltype(x.commDestroy)>(dlsym(lib, "ncclCommDestroy"));
    x.broadcast = reinterpret_cast<decltype(x.broadcast)>(dlsym(lib, "ncclBroadcast"));
    x.groupStart = reinterpret_cast<decltype(x.groupStart)>(dlsym(lib, "ncclGroupStart"));
    x.groupEnd = reinterpret_cast<decltype(x.groupEnd)>(dlsym(lib, "ncclGroupEnd"));
    x.errorString = reinterpret_cast<decltype(x.errorString)>(dlsym(lib, "ncclGetErrorString"));
    x.ok = x.commInitAll && x.commDestroy && x.broadcast && x.groupStart && x.groupEnd && x.errorString;
    return x;
  }();
  return r;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int hfail(hipError_t e, const char* what) {
  set_last_error(std::string(what) + ": " + hipGetErrorString(e));
  return e == hipErrorOutOfMemory ? HIPSPMV_ERR_OOM : HIPSPMV_ERR_HIP;
}

#define MTRY(call)                                  \
  do {                                              \
    hipError_t e_ = (call);                         \
    if (e_ != hipSuccess) return hfail(e_, #call);  \
  } while (0)

float ms_between(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

}  // namespace

struct hipspmv_multi {
  struct Shard {
    int device = 0;
    uint32_t row0 = 0, rows = 0, nnz = 0;
    hipspmv_t* h = nullptr;
    hipStream_t stream = nullptr;
    void *d_x = nullptr, *d_y = nullptr;
    hipEvent_t ev[5] = {};  // start (root) / x on the root (others), x ready, kernel done, y copied,
                            // root only: x ready after the broadcast (its kernel starts there)
    uint64_t kernel_ns = 0;
  };
  std::vector<Shard> shards;
  uint32_t rows = 0, cols = 0, nnz = 0;
  int dtype = HIPSPMV_F64;
  std::vector<ncclComm_t> comms;  // empty: peer copies
  uint64_t setup_ns = 0, h2d_ns = 0, bcast_ns = 0, kernel_ns = 0, d2h_ns = 0, execs = 0;
};

static void release_multi(hipspmv_multi_t* m) {
  if (!m) return;
  for (auto& s : m->shards) {  // released on the library's release thread (capi.cpp defer_release)
    if (s.h) hipspmv_destroy(s.h);
    std::vector<void*> evs(std::begin(s.ev), std::end(s.ev));
    try {
      defer_release(s.device, {s.d_x, s.d_y}, std::move(evs), {s.stream});
    } catch (...) {  // host OOM while queueing: leaked, never freed under a live launch
    }
  }
  for (ncclComm_t c : m->comms) rccl().commDestroy(c);
  delete m;
}

template <class Build>
static int multi_create(uint32_t rows, uint32_t cols, uint32_t nnz, int dtype, const int* devices, int ndev,
                        hipspmv_multi_t** out, Build&& build) {
  if (!out || !devices || ndev < 1 || ndev > 64) return HIPSPMV_ERR_INVALID_ARG;
  *out = nullptr;
  if (dtype != HIPSPMV_F64 && dtype != HIPSPMV_U64) return HIPSPMV_ERR_INVALID_ARG;
  if (rows == 0 || cols == 0) return HIPSPMV_ERR_INVALID_ARG;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    set_last_error("no HIP device");
    return HIPSPMV_ERR_NO_DEVICE;
  }
  for (int i = 0; i < ndev; ++i)
    if (devices[i] < 0 || devices[i] >= count) return HIPSPMV_ERR_NO_DEVICE;
  const auto t0 = std::chrono::steady_clock::now();
  HostCSR a;
  std::string why;
  if (int st = build(a, why)) {
    set_last_error(why);
    return st;
  }
  // cost-balanced contiguous blocks at multiples of HIPSPMV_SHARD_ALIGN, so
  // every kernel gives the single-device bits (include/hipspmv.h)
  std::vector<uint32_t> bounds(ndev + 1, 0);
  partition_rows_cost(a.rowptr.data(), a.colind.data(), rows, (uint32_t)ndev, bounds.data());
  auto* m = new hipspmv_multi;
  m->rows = rows;
  m->cols = cols;
  m->nnz = nnz;
  m->dtype = dtype;
  m->shards.resize(ndev);
  for (int i = 0; i < ndev; ++i) {
    auto& s = m->shards[i];
    s.device = devices[i];
    s.row0 = bounds[i];
    s.rows = bounds[i + 1] - bounds[i];
    const uint32_t e0 = a.rowptr[s.row0], e1 = a.rowptr[s.row0 + s.rows];
    s.nnz = e1 - e0;
    DevGuard g(s.device);
    int st = HIPSPMV_OK;
    if (s.rows) {
      std::vector<uint32_t> rp(s.rows + 1);
      for (uint32_t r = 0; r <= s.rows; ++r) rp[r] = a.rowptr[s.row0 + r] - e0;
      st = hipspmv_create_csr(rp.data(), a.colind.data() + e0, a.vals.data() + e0, s.rows, cols, s.nnz, dtype,
                              s.device, &s.h);
    }
    hipError_t e = hipSuccess;
    if (!st) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    for (int k = 0; k < 5 && !st && e == hipSuccess; ++k) e = hipEventCreate(&s.ev[k]);
    if (!st && e == hipSuccess) e = hipMalloc(&s.d_x, 8ull * cols);
    if (!st && e == hipSuccess) e = hipMalloc(&s.d_y, 8ull * std::max<uint32_t>(s.rows, 1));
    if (!st && e != hipSuccess) st = hfail(e, "multi shard setup");
    if (st) {
      release_multi(m);
      return st;
    }
  }
  // RCCL needs distinct devices; with repeats the broadcast is peer copies
  std::vector<int> devs(devices, devices + ndev);
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (ndev > 1 && distinct && rccl().ok) {
    m->comms.resize(ndev);
    ncclResult_t r = rccl().commInitAll(m->comms.data(), ndev, devs.data());
    if (r != ncclSuccess) {
      m->comms.clear();  // fall back to peer copies (still device to device)
    }
  }
  m->setup_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now() - t0).count();
  *out = m;
  return HIPSPMV_OK;
}

static int multi_exec(hipspmv_multi_t* m, const void* x, void* y, int beta, int mode) {
  if (!m || !x || !y || (beta != 0 && beta != 1)) return HIPSPMV_ERR_INVALID_ARG;
  const size_t bx = 8ull * m->cols;
  auto& root = m->shards[0];
  // 1. x to the root device
  {
    DevGuard g(root.device);
    MTRY(hipEventRecord(root.ev[0], root.stream));
    MTRY(hipMemcpyAsync(root.d_x, x, bx, hipMemcpyHostToDevice, root.stream));
    MTRY(hipEventRecord(root.ev[1], root.stream));
  }
  // 2. broadcast root -> others, ordered after the upload.  ev[0] of a
  //    non-root shard marks "x is on the root" on that shard's own device, so
  //    the broadcast time is measured between two events of one device.
  for (size_t i = 1; i < m->shards.size(); ++i) {
    auto& s = m->shards[i];
    DevGuard g(s.device);
    MTRY(hipStreamWaitEvent(s.stream, root.ev[1], 0));
    MTRY(hipEventRecord(s.ev[0], s.stream));
  }
  if (m->shards.size() > 1) {
    if (!m->comms.empty()) {
      const Rccl& R = rccl();
      R.groupStart();
      ncclResult_t r = ncclSuccess;
      for (size_t i = 0; i < m->shards.size() && r == ncclSuccess; ++i) {
        auto& s = m->shards[i];
        r = R.broadcast(root.d_x, s.d_x, m->cols, m->dtype == HIPSPMV_U64 ? ncclUint64 : ncclFloat64, 0,
                        m->comms[i], s.stream);
      }
      ncclResult_t r2 = R.groupEnd();
      if (r != ncclSuccess || r2 != ncclSuccess) {
        set_last_error(std::string("ncclBroadcast: ") + R.errorString(r != ncclSuccess ? r : r2));
        return HIPSPMV_ERR_HIP;
      }
    } else {
      for (size_t i = 1; i < m->shards.size(); ++i) {
        auto& s = m->shards[i];
        DevGuard g(s.device);
        MTRY(hipMemcpyPeerAsync(s.d_x, s.device, root.d_x, root.device, bx, s.stream));
      }
    }
  }
  for (size_t i = 1; i < m->shards.size(); ++i) {
    auto& s = m->shards[i];
    DevGuard g(s.device);
    MTRY(hipEventRecord(s.ev[1], s.stream));
  }
  {  // the root's own kernel starts after the broadcast it takes part in (RCCL runs on its stream)
    DevGuard g(root.device);
    MTRY(hipEventRecord(root.ev[4], root.stream));
  }
  // 3. per shard: y in (beta 1), kernel, y out
  char* yb = static_cast<char*>(y);
  for (auto& s : m->shards) {
    if (!s.rows) continue;
    DevGuard g(s.device);
    const size_t by = 8ull * s.rows;
    if (beta) MTRY(hipMemcpyAsync(s.d_y, yb + 8ull * s.row0, by, hipMemcpyHostToDevice, s.stream));
    if (int st = hipspmv_exec_device(s.h, s.d_x, s.d_y, s.d_y, beta, mode, s.stream)) return st;
    MTRY(hipEventRecord(s.ev[2], s.stream));
    MTRY(hipMemcpyAsync(yb + 8ull * s.row0, s.d_y, by, hipMemcpyDeviceToHost, s.stream));
    MTRY(hipEventRecord(s.ev[3], s.stream));
  }
  for (auto& s : m->shards) {
    DevGuard g(s.device);
    MTRY(hipStreamSynchronize(s.stream));
  }
  // 4. times: broadcast = root upload done -> x on the device, slowest device; kernel =
  //    slowest shard (its x-ready -> kernel-done, which includes y in for beta 1)
  m->h2d_ns = (uint64_t)(ms_between(root.ev[0], root.ev[1]) * 1e6);
  uint64_t bc = 0, kern = 0, d2h = 0;
  for (size_t i = 0; i < m->shards.size(); ++i) {
    auto& s = m->shards[i];
    if (i > 0) bc = std::max(bc, (uint64_t)(ms_between(s.ev[0], s.ev[1]) * 1e6));
    if (!s.rows) continue;
    s.kernel_ns = (uint64_t)(ms_between(i == 0 ? s.ev[4] : s.ev[1], s.ev[2]) * 1e6);
    kern = std::max(kern, s.kernel_ns);
    d2h = std::max(d2h, (uint64_t)(ms_between(s.ev[2], s.ev[3]) * 1e6));
  }
  m->bcast_ns = bc;
  m->kernel_ns = kern;
  m->d2h_ns = d2h;
  m->execs++;
  return HIPSPMV_OK;
}

extern "C" {

int hipspmv_multi_create(const uint32_t* colptr, const uint32_t* rowind, const void* vals, uint32_t rows,
                         uint32_t cols, uint32_t nnz, int dtype, const int* devices, int ndev,
                         hipspmv_multi_t** out) {
  if (!colptr || (nnz && (!rowind || !vals))) return HIPSPMV_ERR_INVALID_ARG;
  try {
    return multi_create(rows, cols, nnz, dtype, devices, ndev, out, [&](HostCSR& a, std::string& why) {
      return csc_to_csr(colptr, rowind, vals, rows, cols, nnz, a, why);
    });
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    return HIPSPMV_ERR_INVALID_ARG;
  }
}

int hipspmv_multi_create_csr(const uint32_t* rowptr, const uint32_t* colind, const void* vals, uint32_t rows,
                             uint32_t cols, uint32_t nnz, int dtype, const int* devices, int ndev,
                             hipspmv_multi_t** out) {
  if (!rowptr || (nnz && (!colind || !vals))) return HIPSPMV_ERR_INVALID_ARG;
  try {
    return multi_create(rows, cols, nnz, dtype, devices, ndev, out, [&](HostCSR& a, std::string& why) {
      return copy_csr(rowptr, colind, vals, rows, cols, nnz, a, why);
    });
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    return HIPSPMV_ERR_INVALID_ARG;
  }
}

int hipspmv_multi_shard(hipspmv_multi_t* m, int i, hipspmv_t** out) {
  if (!m || !out || i < 0 || (size_t)i >= m->shards.size()) return HIPSPMV_ERR_INVALID_ARG;
  *out = m->shards[i].h;  // NULL for a block without rows
  return HIPSPMV_OK;
}

int hipspmv_partition_rows(const uint32_t* rowptr, const uint32_t* colind, uint32_t rows, uint32_t cols,
                           uint32_t parts, uint32_t* bounds) {
  if (!rowptr || !bounds || parts < 1 || rows == 0) return HIPSPMV_ERR_INVALID_ARG;
  const uint32_t nnz = rowptr[rows];
  if (nnz && !colind) return HIPSPMV_ERR_INVALID_ARG;
  for (uint32_t r = 0; r < rows; ++r)
    if (rowptr[r] > rowptr[r + 1]) return HIPSPMV_ERR_INVALID_MATRIX;
  for (uint32_t e = 0; e < nnz; ++e)
    if (colind[e] >= cols) return HIPSPMV_ERR_INVALID_MATRIX;
  try {
    partition_rows_cost(rowptr, colind, rows, parts, bounds);
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  }
  return HIPSPMV_OK;
}

int hipspmv_multi_set_option(hipspmv_multi_t* m, const char* key, int64_t value) {
  if (!m || !key) return HIPSPMV_ERR_INVALID_ARG;
  for (auto& s : m->shards)
    if (s.h)
      if (int st = hipspmv_set_option(s.h, key, value)) return st;
  return HIPSPMV_OK;
}

int hipspmv_multi_exec(hipspmv_multi_t* m, const void* x, void* y, int beta, int mode) {
  try {
    return multi_exec(m, x, y, beta, mode);
  } catch (const std::bad_alloc&) {
    return HIPSPMV_ERR_OOM;
  } catch (...) {
    set_last_error("unexpected C++ exception");
    return HIPSPMV_ERR_HIP;
  }
}

int hipspmv_multi_stat(hipspmv_multi_t* m, const char* key, uint64_t* out) {
  if (!m || !key || !out) return HIPSPMV_ERR_INVALID_ARG;
  const std::string k(key);
  if (k == "num_devices") *out = m->shards.size();
  else if (k == "rccl") *out = m->comms.empty() ? 0 : 1;
  else if (k == "rows") *out = m->rows;
  else if (k == "cols") *out = m->cols;
  else if (k == "nz") *out = m->nnz;
  else if (k == "setup_ns") *out = m->setup_ns;
  else if (k == "h2d_ns") *out = m->h2d_ns;
  else if (k == "bcast_ns") *out = m->bcast_ns;
  else if (k == "kernel_ns") *out = m->kernel_ns;
  else if (k == "d2h_ns") *out = m->d2h_ns;
  else if (k == "execs") *out = m->execs;
  else if (k == "kernel") {  // the kernel the first non-empty block ran last (HIPSPMV_KERNEL_*)
    uint64_t v = 0;
    for (auto& s : m->shards)  // the first non-empty block (a block of a small matrix may have no rows)
      if (s.h) {
        (void)hipspmv_stat(s.h, "kernel", &v);
        break;
      }
    *out = v;
  }
  else if (k == "total_cycles") {  // the multi-device launch (x ready -> last block done) at block 0's clock
    uint64_t khz = 0;
    for (auto& s : m->shards)
      if (s.h && hipspmv_stat(s.h, "clock_khz", &khz) == HIPSPMV_OK) break;
    *out = (uint64_t)std::ceil(m->kernel_ns * (khz / 1e6));
  } else if (k == "read_misses" || k == "hazard_stalls" || k == "ocm_depth" ||
             k == "active_cycles") {  // summed over blocks (misses, stalls) or the largest block's
    const bool sum = k == "read_misses" || k == "hazard_stalls";
    uint64_t acc = 0;
    for (auto& s : m->shards) {
      uint64_t v = 0;
      if (!s.h) continue;
      if (int st = hipspmv_stat(s.h, key, &v)) return st;
      acc = sum ? acc + v : std::max(acc, v);
    }
    *out = acc;
  } else if (k.rfind("state_", 0) == 0 || k == "no_valid_but_ready" || k == "no_ready_but_valid" ||
             k == "profiled" || k == "profile" || k == "profile_units" || k == "profile_span_cycles" ||
             k == "issue_window" || k == "capacity_stalls" || k == "cms") {
    // NewCache state statistics: the slowest block's (max); "profiled" only
    // if every block's last launch was profiled (min); units summed
    const bool mn = k == "profiled" || k == "profile", sum = k == "profile_units";
    uint64_t acc = mn ? 1 : 0;
    bool any = false;
    for (auto& s : m->shards) {
      uint64_t v = 0;
      if (!s.h) continue;
      if (int st = hipspmv_stat(s.h, key, &v)) return st;
      acc = mn ? std::min(acc, v) : sum ? acc + v : std::max(acc, v);
      any = true;
    }
    *out = any ? acc : 0;
  } else if (k == "alg_bytes") {
    // per device: its rows' entries + its rowptr + all of x + its y
    uint64_t b = 0;
    for (auto& s : m->shards) b += 12ull * s.nnz + 4ull * (s.rows + 1ull) + 8ull * m->cols + 8ull * s.rows;
    *out = b;
  } else if (k.rfind("shard", 0) == 0) {
    // shard<i>_{rows,row0,nz,device,kernel_ns}
    const size_t us = k.find('_');
    if (us == std::string::npos) return HIPSPMV_ERR_KEY;
    const size_t i = std::strtoul(k.substr(5, us - 5).c_str(), nullptr, 10);
    if (i >= m->shards.size()) return HIPSPMV_ERR_KEY;
    const std::string f = k.substr(us + 1);
    const auto& s = m->shards[i];
    if (f == "rows") *out = s.rows;
    else if (f == "row0") *out = s.row0;
    else if (f == "nz") *out = s.nnz;
    else if (f == "device") *out = (uint64_t)s.device;
    else if (f == "kernel_ns") *out = s.kernel_ns;
    else return HIPSPMV_ERR_KEY;
  } else {
    return HIPSPMV_ERR_KEY;
  }
  return HIPSPMV_OK;
}

int hipspmv_multi_destroy(hipspmv_multi_t* m) {
  if (!m) return HIPSPMV_ERR_INVALID_ARG;
  release_multi(m);
  return HIPSPMV_OK;
}

}  // extern "C"
