// Live MI355X telemetry for the node's metrics endpoint: GFX / HBM-controller
// activity, socket power, temperatures, the clock the GPU holds, energy, per-link xGMI traffic and
// power/thermal throttle residency — read from the SMU's gpu_metrics table through AMD SMI.
//
// libamd_smi is dlopen'ed on first use, so the control plane runs on nodes without ROCm (every
// call then reports "unavailable"). KFAMD_SMI_FAKE=<json file> replaces the library with a fixed
// table (CPU tests): {"devices": [{"bdf": "0000:05:00.0", "gfx_activity": 97, ...}]}.
#pragma once

#include <array>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace kf {

struct GpuTelemetry {
  std::string bdf;               // "0000:05:00.0" (GpuDevice::pci_bus)
  double gfx_activity = -1;      // %
  double umc_activity = -1;      // % (HBM memory controllers)
  double power_w = -1;           // socket power
  double temp_hotspot_c = -1;
  double temp_mem_c = -1;
  double gfxclk_mhz = -1;        // current GFX clock (XCC 0): the clock the chip holds under load
  double energy_j = -1;          // accumulated since driver load
  std::array<double, 8> xgmi_read_bytes{};   // accumulated, per link
  std::array<double, 8> xgmi_write_bytes{};
  int xgmi_links = 0;            // links with data (0: no xGMI counters on this part)
  uint64_t accumulation_counter = 0;         // SMU accumulation ticks (throttle residency base)
  uint64_t ppt_residency_acc = 0;            // ticks spent power-limited (PVIOL)
  uint64_t thermal_residency_acc = 0;        // ticks spent thermally limited (TVIOL)
};

class AmdSmi {
 public:
  static AmdSmi& instance();
  // one sample of every GPU the library sees; empty when unavailable
  std::vector<GpuTelemetry> sample();
  bool available();
  std::string error();

 private:
  AmdSmi() = default;
  bool load_locked();
  std::mutex mu_;
  bool tried_ = false, ok_ = false;
  std::string err_, fake_path_;
  void* lib_ = nullptr;
  void* fn_[6] = {};
};

// "0000:05:00.0" from the PCI fields
std::string format_bdf(uint64_t domain, unsigned bus, unsigned device, unsigned function);

}  // namespace kf
