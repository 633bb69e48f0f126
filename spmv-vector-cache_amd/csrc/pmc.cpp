// Hardware counters behind the NewCache statistics.
//
// The reference reads its cache statistics from hardware after every run
// (software/HardwareSpMVNewCache.cpp:161-173, 189-204: readMisses,
// hazardStalls, ...).  The GPU's counters are read by rocprofv3 in separate
// --pmc passes, so the values come from the counter CSV of such a run:
// hipspmv_pmc_counter() returns a counter's mean per dispatch over the
// dispatches of one kernel in a rocprofv3 counter_collection.csv (or the
// value column of a tools/pmc_summary.py summary).  No HIP call: it works on
// a host without a GPU.
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "hipspmv.h"
#include "hipspmv_internal.h"

namespace {

// one CSV record; quoted fields may hold commas ("void k<double, 3>(...)")
// and doubled quotes
bool csv_fields(const std::string& line, std::vector<std::string>& out) {
  out.clear();
  std::string f;
  bool q = false;
  for (size_t i = 0; i < line.size(); ++i) {
    const char c = line[i];
    if (q) {
      if (c == '"' && i + 1 < line.size() && line[i + 1] == '"') {
        f += '"';
        ++i;
      } else if (c == '"') {
        q = false;
      } else {
        f += c;
      }
    } else if (c == '"') {
      q = true;
    } else if (c == ',') {
      out.push_back(f);
      f.clear();
    } else if (c != '\r') {
      f += c;
    }
  }
  out.push_back(f);
  return !q;
}

}  // namespace

extern "C" int hipspmv_pmc_counter(const char* csv_path, const char* kernel, const char* counter, double* mean,
                                   uint64_t* dispatches) {
  if (!csv_path || !counter || !mean) return HIPSPMV_ERR_INVALID_ARG;
  *mean = 0.0;
  if (dispatches) *dispatches = 0;
  try {
    std::ifstream in(csv_path);
    if (!in) {
      hipspmv::set_last_error(std::string("pmc: cannot open ") + csv_path);
      return HIPSPMV_ERR_INVALID_ARG;
    }
    std::string line;
    std::vector<std::string> f, head;
    if (!std::getline(in, line) || !csv_fields(line, head)) return HIPSPMV_ERR_INVALID_MATRIX;
    auto col = [&](const char* name) {
      for (size_t i = 0; i < head.size(); ++i)
        if (head[i] == name) return (int)i;
      return -1;
    };
    const int c_name = col("Counter_Name"), c_val = col("Counter_Value"), c_kern = col("Kernel_Name"),
              c_disp = col("Dispatch_Id");
    if (c_name < 0) {  // tools/pmc_summary.py: counter, dispatches, per_dispatch, per_cu
      const int s_name = col("counter"), s_disp = col("dispatches"), s_val = col("per_dispatch");
      if (s_name < 0 || s_val < 0) {
        hipspmv::set_last_error("pmc: neither a counter_collection nor a pmc_summary CSV");
        return HIPSPMV_ERR_INVALID_MATRIX;
      }
      while (std::getline(in, line)) {
        if (!csv_fields(line, f) || (int)f.size() <= s_val || f[s_name] != counter) continue;
        *mean = std::stod(f[s_val]);
        if (dispatches && s_disp >= 0 && !f[s_disp].empty()) *dispatches = std::stoull(f[s_disp]);
        return HIPSPMV_OK;
      }
      return HIPSPMV_ERR_KEY;
    }
    if (c_val < 0 || c_kern < 0) return HIPSPMV_ERR_INVALID_MATRIX;
    // per matching kernel name: the counter's value per dispatch; the kernel
    // with the most dispatches wins (one CSV may hold several instantiations)
    std::map<std::string, std::map<std::string, double>> per;  // kernel -> dispatch -> value
    const std::string want = kernel ? kernel : "hipspmv::";
    size_t row = 0;
    while (std::getline(in, line)) {
      ++row;
      if (!csv_fields(line, f) || (int)f.size() <= std::max(c_val, std::max(c_name, c_kern))) continue;
      if (f[c_name] != counter || f[c_kern].find(want) == std::string::npos) continue;
      const std::string d = c_disp >= 0 ? f[c_disp] : std::to_string(row);
      per[f[c_kern]][d] += std::stod(f[c_val]);  // a counter split over instances sums per dispatch
    }
    const std::map<std::string, double>* best = nullptr;
    for (const auto& kv : per)
      if (!best || kv.second.size() > best->size()) best = &kv.second;
    if (!best || best->empty()) return HIPSPMV_ERR_KEY;
    double s = 0;
    for (const auto& kv : *best) s += kv.second;
    *mean = s / (double)best->size();
    if (dispatches) *dispatches = best->size();
    return HIPSPMV_OK;
  } catch (...) {
    hipspmv::set_last_error("pmc: malformed counter CSV");
    return HIPSPMV_ERR_INVALID_MATRIX;
  }
}
