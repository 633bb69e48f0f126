// HIPSpMV: the MI355X backend registered in HWSpMVFactory.
//
// Replaces the FPGA backends (software/HardwareSpMV{BufferAll,BufferNone,
// BufferSel,NewCache}.cpp) and the Chisel SpMVAccelerator* RTL behind them.
// It keeps the reference's exec() phase sequence (HardwareSpMVNewCache.cpp:
// 78-88: reset -> setupRegs -> init -> regular -> write) and drives
// libhipspmv.so through the C ABI of include/hipspmv.h.
#ifndef SPMV_AMD_HIPSPMV_H_
#define SPMV_AMD_HIPSPMV_H_

#include <cstdint>
#include <string>

#include "HardwareSpMV.h"
#include "hipspmv.h"

struct hipspmv_handle;
struct hipspmv_multi;

// The in-memory register block that stands in for the accelerator's AXI-Lite
// register map: word 0 is the signature HWSpMVFactory dispatches on
// (cf. SpMVAcceleratorNewCacheDriver.hpp:6 expSignature()).
struct HIPSpMVRegisterFile {
  uint32_t signature;
  int32_t device;  // HIP device ordinal
  int32_t mode;    // HIPSPMV_MODE_* (ORDERED: bit-exact vs SoftwareSpMV)
  int32_t kernel;  // HIPSPMV_KERNEL_* (AUTO picks by matrix shape)
  int32_t beta;    // 1: y += A*x (reference semantics), 0: y = A*x
  uint32_t reset;  // the reset word resetAccelerator() pulses
  // > 1: rows partitioned over devices[0..num_devices) of this process
  // (hipspmv_multi_*; x broadcast device to device).  0 or 1: `device` alone.
  int32_t num_devices;
  int32_t devices[16];
  // 1: vcache-family launches record the NewCache state statistics (sActive,
  // sFill, ..., noValidButReady) -- the reference's profileSel/profileCount
  // registers (SpMVAcceleratorNewCache.scala:44,58) read after the run
  int32_t profile;
};

class HIPSpMV : public HardwareSpMV {
 public:
  static constexpr uint32_t kSignature = 0x4D493335u;  // "MI35"
  static uint32_t expSignature() { return kSignature; }
  // A register block per device, initialised to (device, ORDERED, AUTO, beta 1).
  static HIPSpMVRegisterFile* registerFile(int device = 0);

  HIPSpMV(uintptr_t aBase, uintptr_t aReset, SparseMatrix* A, SpMVData* x, SpMVData* y);
  virtual ~HIPSpMV();

  // One synchronous y (+)= A*x; returns true on success (the FPGA backends
  // always returned false and main.cpp:245 ignores it).  On failure
  // statInt("error") holds the HIPSPMV_* status.
  virtual bool exec();

  virtual unsigned int statInt(std::string name);
  virtual std::vector<std::string> statKeys();
  uint64_t statU64(const std::string& key);  // full-width libhipspmv statistic
  int status() const { return m_status; }
  // A rocprofv3 --pmc counter CSV of this backend's kernel: readMisses,
  // hazardStalls and capacityStalls then report the measured counters
  // (TCC_MISS, SQ_LDS_BANK_CONFLICT, TCP_PENDING_STALL_CYCLES per launch), as
  // the reference reads its counters from the accelerator
  // (HardwareSpMVNewCache.cpp:161-173); readMissesModel / hazardStallsModel
  // keep the layout values.  "" detaches.
  void setPmcCsv(const std::string& path);

 protected:
  const HIPSpMVRegisterFile* regs() const { return reinterpret_cast<const HIPSpMVRegisterFile*>(
                                                const_cast<const uint32_t*>(m_accelBase)); }
  virtual void setupRegs();
  virtual void init();
  virtual void regular();
  virtual void write();
  virtual void setThresholdRegisters();

  const hipspmv_prep_stats_t& prepStats();

  bool multi() const { return regs()->num_devices > 1; }

  hipspmv_handle* m_h = nullptr;
  hipspmv_multi* m_multi = nullptr;
  hipspmv_prep_stats_t m_prep{};
  uint64_t m_prepVersion = ~0ull;
  uint64_t m_builtVersion = ~0ull;
  int m_status = 0;
  std::string m_pmc;
};

#endif
