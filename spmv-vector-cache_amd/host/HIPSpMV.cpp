#include "HIPSpMV.h"

#include <iostream>
#include <map>
#include <mutex>

#include "hipspmv.h"

HIPSpMVRegisterFile* HIPSpMV::registerFile(int device) {
  static std::mutex mu;
  static std::map<int, HIPSpMVRegisterFile> files;
  std::lock_guard<std::mutex> lock(mu);
  auto it = files.find(device);
  if (it == files.end())
    it = files.emplace(device, HIPSpMVRegisterFile{kSignature, device, HIPSPMV_MODE_ORDERED, HIPSPMV_KERNEL_AUTO, 1, 0,
                                                   1, {device}, 0})
             .first;
  return &it->second;
}

HIPSpMV::HIPSpMV(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y)
    : HardwareSpMV(aBase, aReset, A, x, y) {}

HIPSpMV::~HIPSpMV() {
  if (m_h) hipspmv_destroy(m_h);
  if (m_multi) hipspmv_multi_destroy(m_multi);
}

// setupRegs(): the device copy of A is built once per matrix version (CSC ->
// CSR transpose, kernel layouts, upload) and reused by later exec() calls --
// the analogue of programming the base-address registers
// (HardwareSpMVNewCache.cpp:31-44) without re-sending the matrix.
void HIPSpMV::setupRegs() {
  HardwareSpMV::setupRegs();
  if (m_status) return;
  const bool built = multi() ? m_multi != nullptr : m_h != nullptr;
  if (built && m_builtVersion == m_A->version()) return;
  if (m_h) {
    hipspmv_destroy(m_h);
    m_h = nullptr;
  }
  if (m_multi) {
    hipspmv_multi_destroy(m_multi);
    m_multi = nullptr;
  }
  const int dtype = m_A->getDataType() == SPMV_U64 ? HIPSPMV_U64 : HIPSPMV_F64;
  if (multi()) {
    const int n = regs()->num_devices < 16 ? regs()->num_devices : 16;
    m_status = hipspmv_multi_create(m_A->getIndPtrs(), m_A->getInds(), m_A->getNzData(), m_A->getRows(),
                                    m_A->getCols(), m_A->getNz(), dtype, regs()->devices, n, &m_multi);
  } else {
    m_status = hipspmv_create(m_A->getIndPtrs(), m_A->getInds(), m_A->getNzData(), m_A->getRows(), m_A->getCols(),
                              m_A->getNz(), dtype, regs()->device, &m_h);
  }
  if (m_status) {
    std::cerr << "HIPSpMV: create failed: " << hipspmv_strerror(m_status) << " (" << hipspmv_last_error() << ")"
              << std::endl;
    m_h = nullptr;
    m_multi = nullptr;
    return;
  }
  m_builtVersion = m_A->version();
  if (m_h && !m_pmc.empty()) hipspmv_attach_pmc(m_h, m_pmc.c_str());
  if (regs()->kernel != HIPSPMV_KERNEL_AUTO)
    m_status = multi() ? hipspmv_multi_set_option(m_multi, "kernel", regs()->kernel)
                       : hipspmv_set_option(m_h, "kernel", regs()->kernel);
}

void HIPSpMV::init() {}

// regular(): x to the device, the kernel, y back -- synchronously, like the
// reference's busy-wait on doneRegular (HardwareSpMVNewCache.cpp:90-101).
void HIPSpMV::regular() {
  if (m_status || !(m_h || m_multi)) return;
  m_status = m_multi ? hipspmv_multi_set_option(m_multi, "profile", regs()->profile)
                     : hipspmv_set_option(m_h, "profile", regs()->profile);
  if (m_status) return;
  m_status = m_multi ? hipspmv_multi_exec(m_multi, m_x, m_y, regs()->beta, regs()->mode)
                     : hipspmv_exec(m_h, m_x, m_y, regs()->beta, regs()->mode);
  if (m_status)
    std::cerr << "HIPSpMV: exec failed: " << hipspmv_strerror(m_status) << " (" << hipspmv_last_error() << ")"
              << std::endl;
}

void HIPSpMV::write() {}

// There are no stream FIFOs to throttle; the thresholds are kept only so
// setThresholds() stays callable and they appear in the statistics.
void HIPSpMV::setThresholdRegisters() {}

bool HIPSpMV::exec() {
  m_status = 0;
  resetAccelerator();
  setupRegs();
  init();
  regular();
  write();
  return m_status == 0;
}

void HIPSpMV::setPmcCsv(const std::string& path) {
  m_pmc = path;
  if (m_h) hipspmv_attach_pmc(m_h, path.c_str());
}

uint64_t HIPSpMV::statU64(const std::string& key) {
  uint64_t v = 0;
  if (m_multi) {
    if (key == "alg_bytes_beta1") {  // y read as well
      if (hipspmv_multi_stat(m_multi, "alg_bytes", &v) == HIPSPMV_OK) return v + 8ull * m_A->getRows();
      return 0;
    }
    return hipspmv_multi_stat(m_multi, key.c_str(), &v) == HIPSPMV_OK ? v : 0;
  }
  if (m_h && hipspmv_stat(m_h, key.c_str(), &v) == HIPSPMV_OK) return v;
  if (key == "num_devices") return 1;
  return 0;
}

std::vector<std::string> HIPSpMV::statKeys() {
  std::vector<std::string> keys = HardwareSpMV::statKeys();
  for (const char* k : {"kernelTimeUs", "setupTimeUs", "h2dTimeUs", "d2hTimeUs", "algKBytes", "mode", "kernel",
                        "device", "error", "numDevices", "bcastTimeUs", "maxAlive", "maxColSpan", "cmstime",
                        "maxAliveTime", "maxColSpanTime"})
    keys.push_back(k);
  // HardwareSpMVNewCache::statKeys (HardwareSpMVNewCache.cpp:189-204), same names and order
  for (const char* k : {"sActive", "sFill", "sFlush", "sDone", "sReadMiss1", "sReadMiss2", "sReadMiss3",
                        "sColdMiss", "totalCycles", "activeCycles", "readMisses", "ocmDepth", "issueWindow",
                        "hazardStalls", "capacityStalls", "cms", "noValidButReady", "noReadyButValid"})
    keys.push_back(k);
  // the layout-derived values readMisses / hazardStalls report without a counter CSV
  for (const char* k : {"readMissesModel", "hazardStallsModel"}) keys.push_back(k);
  return keys;
}

// The SoftwareSpMV preprocessing statistics (SoftwareSpMV.cpp:72-95), computed
// on the GPU once per matrix version (hipspmv_prep_stats); times in us.
const hipspmv_prep_stats_t& HIPSpMV::prepStats() {
  if (m_prepVersion != m_A->version()) {
    m_prep = hipspmv_prep_stats_t{};
    int st = hipspmv_prep_stats(m_A->getIndPtrs(), m_A->getInds(), m_A->getRows(), m_A->getCols(), m_A->getNz(),
                                regs()->device, &m_prep);
    if (st)
      std::cerr << "HIPSpMV: prep_stats failed: " << hipspmv_strerror(st) << " (" << hipspmv_last_error() << ")"
                << std::endl;
    m_prepVersion = m_A->version();
  }
  return m_prep;
}

unsigned int HIPSpMV::statInt(std::string name) {
  if (name == "kernelTimeUs") return (unsigned int)(statU64("kernel_ns") / 1000);
  if (name == "setupTimeUs") return (unsigned int)(statU64("setup_ns") / 1000);
  if (name == "h2dTimeUs") return (unsigned int)(statU64("h2d_ns") / 1000);
  if (name == "d2hTimeUs") return (unsigned int)(statU64("d2h_ns") / 1000);
  if (name == "algKBytes") return (unsigned int)(statU64(regs()->beta ? "alg_bytes_beta1" : "alg_bytes") / 1024);
  if (name == "mode") return (unsigned int)regs()->mode;
  if (name == "kernel") return (unsigned int)statU64("kernel");
  if (name == "device") return (unsigned int)regs()->device;
  if (name == "error") return (unsigned int)m_status;
  if (name == "numDevices") return (unsigned int)statU64("num_devices");
  if (name == "bcastTimeUs") return (unsigned int)(statU64("bcast_ns") / 1000);
  if (name == "maxAlive") return prepStats().max_alive;
  if (name == "maxColSpan") return prepStats().max_col_span;
  if (name == "cmstime") return (unsigned int)(prepStats().cms_ns / 1000);
  if (name == "maxAliveTime") return (unsigned int)(prepStats().max_alive_ns / 1000);
  if (name == "maxColSpanTime") return (unsigned int)(prepStats().max_col_span_ns / 1000);
  // the reference's cache-behaviour keys (HardwareSpMVNewCache.cpp:189-204), for the last launch:
  // totalCycles = kernel time x shader clock; activeCycles = the cycles it would take at the HBM
  // roofline (activeCycles / totalCycles = roofline fraction, the reference's Active/Total);
  // readMisses = x words not on chip when a product needed them (streamed into the LDS cache, or
  // gathered from L2/HBM); hazardStalls = adds that waited on the previous add to their y row;
  // ocmDepth = on-chip vector-cache words per workgroup (y block + x panels)
  if (name == "totalCycles") return (unsigned int)statU64("total_cycles");
  if (name == "activeCycles") return (unsigned int)statU64("active_cycles");
  // with a counter CSV and no device handle (the run failed, or the CSV comes from another host),
  // the counters still reach the row: the CSV's dominant hipspmv kernel
  if (!m_pmc.empty() && !m_h && !m_multi &&
      (name == "readMisses" || name == "hazardStalls" || name == "capacityStalls")) {
    const char* c = name == "readMisses" ? "TCC_MISS" : name == "hazardStalls" ? "SQ_LDS_BANK_CONFLICT"
                                                                             : "TCP_PENDING_STALL_CYCLES";
    double v = 0;
    uint64_t n = 0;
    if (hipspmv_pmc_counter(m_pmc.c_str(), nullptr, c, &v, &n) == HIPSPMV_OK && n) return (unsigned int)(v + 0.5);
  }
  if (name == "readMisses") return (unsigned int)statU64("read_misses");
  if (name == "hazardStalls") return (unsigned int)statU64("hazard_stalls");
  if (name == "readMissesModel") return (unsigned int)statU64("read_misses_model");
  if (name == "hazardStallsModel") return (unsigned int)statU64("hazard_stalls_model");
  if (name == "ocmDepth") return (unsigned int)statU64("ocm_depth");
  // the cache-FSM state counts (stateNames, HardwareSpMVNewCache.cpp:6-7) and the
  // stream-monitor stalls, measured by a profiled launch (register `profile`):
  // cycles per workgroup (one vector cache), DESIGN.md §6.9
  static const std::map<std::string, const char*> states = {
      {"sActive", "state_active"},         {"sFill", "state_fill"},
      {"sFlush", "state_flush"},           {"sDone", "state_done"},
      {"sReadMiss1", "state_read_miss1"},  {"sReadMiss2", "state_read_miss2"},
      {"sReadMiss3", "state_read_miss3"},  {"sColdMiss", "state_cold_miss"},
      {"issueWindow", "issue_window"},     {"capacityStalls", "capacity_stalls"},
      {"cms", "cms"},                      {"noValidButReady", "no_valid_but_ready"},
      {"noReadyButValid", "no_ready_but_valid"}};
  auto it = states.find(name);
  if (it != states.end()) return (unsigned int)statU64(it->second);
  if (name == "thresColPtr") return m_thres.colPtr;
  if (name == "thresRowInd") return m_thres.rowInd;
  if (name == "thresNZData") return m_thres.nzData;
  if (name == "thresInputVec") return m_thres.inpVec;
  return HardwareSpMV::statInt(name);
}
