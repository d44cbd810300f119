#include "gpu/smi.h"

#include <dlfcn.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>

#include "core/json.h"
#include "core/util.h"

// Struct layouts (amdsmi_gpu_metrics_t, amdsmi_bdf_t) and the status/flag constants come from the
// ROCm headers the node image is built against; only the entry points are resolved at run time.
// A build host without ROCm headers gets the fake-table path only.
#if __has_include(<amd_smi/amdsmi.h>)
#include <amd_smi/amdsmi.h>
#define KFAMD_HAVE_AMDSMI 1
#endif

namespace kf {

#ifdef KFAMD_HAVE_AMDSMI
namespace {
using InitFn = amdsmi_status_t (*)(uint64_t);
using SocketsFn = amdsmi_status_t (*)(uint32_t*, amdsmi_socket_handle*);
using ProcsFn = amdsmi_status_t (*)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
using BdfFn = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_bdf_t*);
using MetricsFn = amdsmi_status_t (*)(amdsmi_processor_handle, amdsmi_gpu_metrics_t*);
using ShutFn = amdsmi_status_t (*)();
enum { kInit, kSockets, kProcs, kBdf, kMetrics, kShut };

// gpu_metrics fields the SMU does not fill read as all-ones
template <typename T>
double valid(T v, double scale = 1.0) {
  return v == static_cast<T>(~T(0)) ? -1.0 : static_cast<double>(v) * scale;
}
}  // namespace
#endif

std::string format_bdf(uint64_t domain, unsigned bus, unsigned device, unsigned function) {
  char b[32];
  std::snprintf(b, sizeof b, "%04llx:%02x:%02x.%x", static_cast<unsigned long long>(domain), bus, device, function);
  return b;
}

AmdSmi& AmdSmi::instance() {
  static AmdSmi s;
  return s;
}

bool AmdSmi::load_locked() {
  if (tried_) return ok_;
  tried_ = true;
  if (const char* f = std::getenv("KFAMD_SMI_FAKE")) {
    fake_path_ = f;
    ok_ = true;
    return ok_;
  }
#ifndef KFAMD_HAVE_AMDSMI
  err_ = "built without AMD SMI headers";
  return false;
#else
  // Only the SONAME of the headers this file was compiled against: amdsmi_gpu_metrics_t / amdsmi_bdf_t
  // are laid out by those headers, and a library of another major version could write a larger
  // struct into our stack objects. The runtime version is checked as well.
#define KFAMD_STR2(x) #x
#define KFAMD_STR(x) KFAMD_STR2(x)
  const std::string soname = "libamd_smi.so." KFAMD_STR(AMDSMI_LIB_VERSION_MAJOR);
  for (const std::string& name : {soname, std::string("/opt/rocm/lib/") + soname}) {
    lib_ = dlopen(name.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (lib_) break;
  }
#undef KFAMD_STR
#undef KFAMD_STR2
  if (!lib_) {
    const char* e = dlerror();
    err_ = e ? e : (soname + " not found");
    return false;
  }
  if (auto ver = reinterpret_cast<amdsmi_status_t (*)(amdsmi_version_t*)>(dlsym(lib_, "amdsmi_get_lib_version"))) {
    amdsmi_version_t v{};
    if (ver(&v) == AMDSMI_STATUS_SUCCESS && v.major != AMDSMI_LIB_VERSION_MAJOR) {
      err_ = "libamd_smi major version " + std::to_string(v.major) + " != headers' " +
             std::to_string(AMDSMI_LIB_VERSION_MAJOR);
      return false;
    }
  }
  const char* names[] = {"amdsmi_init", "amdsmi_get_socket_handles", "amdsmi_get_processor_handles",
                         "amdsmi_get_gpu_device_bdf", "amdsmi_get_gpu_metrics_info", "amdsmi_shut_down"};
  for (int i = 0; i < 6; ++i) {
    fn_[i] = dlsym(lib_, names[i]);
    if (!fn_[i]) {
      err_ = std::string("missing symbol ") + names[i];
      return false;
    }
  }
  const amdsmi_status_t st = reinterpret_cast<InitFn>(fn_[kInit])(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    err_ = "amdsmi_init failed: " + std::to_string(static_cast<int>(st));
    return false;
  }
  ok_ = true;
  return ok_;
#endif
}

bool AmdSmi::available() {
  std::lock_guard<std::mutex> g(mu_);
  return load_locked();
}

std::string AmdSmi::error() {
  std::lock_guard<std::mutex> g(mu_);
  load_locked();
  return err_;
}

std::vector<GpuTelemetry> AmdSmi::sample() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<GpuTelemetry> out;
  if (!load_locked()) return out;

  if (!fake_path_.empty()) {
    std::string text;
    if (!read_file(fake_path_, text)) return out;
    try {
      const Json j = Json::parse(text);
      for (const auto& d : j["devices"].as_array()) {
        GpuTelemetry t;
        t.bdf = d["bdf"].as_string();
        t.gfx_activity = d["gfx_activity"].as_double(-1);
        t.umc_activity = d["umc_activity"].as_double(-1);
        t.power_w = d["power_w"].as_double(-1);
        t.temp_hotspot_c = d["temp_hotspot_c"].as_double(-1);
        t.temp_mem_c = d["temp_mem_c"].as_double(-1);
        t.gfxclk_mhz = d["gfxclk_mhz"].as_double(-1);
        t.energy_j = d["energy_j"].as_double(-1);
        const auto& rd = d["xgmi_read_bytes"].as_array();
        const auto& wr = d["xgmi_write_bytes"].as_array();
        for (size_t i = 0; i < rd.size() && i < 8; ++i) t.xgmi_read_bytes[i] = rd[i].as_double();
        for (size_t i = 0; i < wr.size() && i < 8; ++i) t.xgmi_write_bytes[i] = wr[i].as_double();
        t.xgmi_links = static_cast<int>(std::min<size_t>(8, std::max(rd.size(), wr.size())));
        t.accumulation_counter = static_cast<uint64_t>(d["accumulation_counter"].as_double());
        t.ppt_residency_acc = static_cast<uint64_t>(d["ppt_residency_acc"].as_double());
        t.thermal_residency_acc = static_cast<uint64_t>(d["thermal_residency_acc"].as_double());
        out.push_back(t);
      }
    } catch (const std::exception&) {
    }
    return out;
  }

#ifdef KFAMD_HAVE_AMDSMI
  uint32_t nsock = 0;
  if (reinterpret_cast<SocketsFn>(fn_[kSockets])(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS || nsock == 0) return out;
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (reinterpret_cast<SocketsFn>(fn_[kSockets])(&nsock, socks.data()) != AMDSMI_STATUS_SUCCESS) return out;
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    if (reinterpret_cast<ProcsFn>(fn_[kProcs])(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> procs(np);
    if (reinterpret_cast<ProcsFn>(fn_[kProcs])(socks[s], &np, procs.data()) != AMDSMI_STATUS_SUCCESS) continue;
    for (uint32_t p = 0; p < np; ++p) {
      amdsmi_bdf_t bdf{};
      if (reinterpret_cast<BdfFn>(fn_[kBdf])(procs[p], &bdf) != AMDSMI_STATUS_SUCCESS) continue;
      amdsmi_gpu_metrics_t m{};
      if (reinterpret_cast<MetricsFn>(fn_[kMetrics])(procs[p], &m) != AMDSMI_STATUS_SUCCESS) continue;
      GpuTelemetry t;
      t.bdf = format_bdf(bdf.domain_number, static_cast<unsigned>(bdf.bus_number), static_cast<unsigned>(bdf.device_number),
                         static_cast<unsigned>(bdf.function_number));
      t.gfx_activity = valid(m.average_gfx_activity);
      t.umc_activity = valid(m.average_umc_activity);
      t.power_w = valid(m.current_socket_power);
      if (t.power_w < 0) t.power_w = valid(m.average_socket_power);
      t.temp_hotspot_c = valid(m.temperature_hotspot);
      t.temp_mem_c = valid(m.temperature_mem);
      t.gfxclk_mhz = valid(m.current_gfxclks[0]);
      if (t.gfxclk_mhz < 0) t.gfxclk_mhz = valid(m.current_gfxclk);
      t.energy_j = valid(m.energy_accumulator, 15.259e-6);  // 15.259 uJ units
      for (int i = 0; i < 8; ++i) {
        const double r = valid(m.xgmi_read_data_acc[i], 1024.0), w = valid(m.xgmi_write_data_acc[i], 1024.0);
        t.xgmi_read_bytes[i] = r < 0 ? 0 : r;
        t.xgmi_write_bytes[i] = w < 0 ? 0 : w;
        if (r >= 0 || w >= 0) t.xgmi_links = i + 1;
      }
      t.accumulation_counter = m.accumulation_counter == ~0ULL ? 0 : m.accumulation_counter;
      t.ppt_residency_acc = m.ppt_residency_acc == ~0ULL ? 0 : m.ppt_residency_acc;
      t.thermal_residency_acc = m.socket_thm_residency_acc == ~0ULL ? 0 : m.socket_thm_residency_acc;
      out.push_back(t);
    }
  }
#endif
  return out;
}

}  // namespace kf
