// util.h — small shared helpers: strings, time (RFC 3339), randomness, files, structured logging.
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <optional>
#include <string>
#include <vector>

#include "core/json.h"

namespace kf {

// ---- strings ---------------------------------------------------------------------------------
std::vector<std::string> split(const std::string& s, char sep, bool skip_empty = false);
std::string join(const std::vector<std::string>& parts, const std::string& sep);
std::string trim(const std::string& s);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
bool contains(const std::string& s, const std::string& p);
std::string to_lower(std::string s);
std::string to_upper(std::string s);
std::string replace_all(std::string s, const std::string& from, const std::string& to);
std::string url_decode(const std::string& s);  // form encoding (queries): '+' is a space
// a request path: percent-decoding only ('+' stays '+')
std::string url_decode_path(const std::string& s);
// an encoded '/' or '\' (%2F, %5C) in a raw path: the gateway refuses these (Istio's REJECT_REQUEST
// for escaped slashes) rather than let routing and authorization disagree on segments
bool path_has_escaped_slash(const std::string& raw_path);
std::string url_encode(const std::string& s);
std::string base64_encode(const std::string& in);
std::string base64_decode(const std::string& in);
std::string random_hex(size_t nbytes);
// credentials (tokens, cookie secrets): getrandom(2), never the PRNG behind random_hex
std::string secure_random_hex(size_t nbytes);
std::string random_alnum(size_t n);
std::string uuid4();
// Kubernetes resource quantities ("500m", "1Gi", "2", "1e3") -> value in base units
// (cores for CPU-like, bytes for memory-like). Returns nullopt on parse failure.
std::optional<double> parse_quantity(const std::string& q);
std::string format_quantity_int(int64_t v);

// ---- time -----------------------------------------------------------------------------------
int64_t now_unix_ms();
double now_seconds();
// Name the calling thread (<= 15 chars, truncated) so per-thread CPU shows in /proc/<pid>/task/*/comm.
void set_thread_name(const std::string& name);  // monotonic
std::string rfc3339_now();                 // second precision, "Z" (Kubernetes metav1.Time)
std::string rfc3339_ms_now();              // millisecond precision (MicroTime-like)
std::string rfc3339_from_ms(int64_t unix_ms, bool with_ms = false);
std::optional<int64_t> parse_rfc3339_ms(const std::string& s);  // -> unix ms

// ---- files ----------------------------------------------------------------------------------
bool read_file(const std::string& path, std::string& out);
bool write_file(const std::string& path, const std::string& data);  // atomic (tmp + rename)
bool file_exists(const std::string& path);
bool make_dirs(const std::string& path);
int64_t file_mtime_ns(const std::string& path);  // -1 if missing
std::string getenv_or(const char* name, const std::string& def);
bool env_true(const char* name, bool def = false);

// ---- logging (zap-like: one JSON object per line, or console) ---------------------------------
enum class LogLevel { Debug = 0, Info = 1, Warn = 2, Error = 3 };
class Logger {
 public:
  static Logger& get();
  void set_level(LogLevel l) { level_ = l; }
  void set_json(bool j) { json_ = j; }
  void set_sink(std::function<void(const std::string&)> sink);
  bool enabled(LogLevel l) const { return static_cast<int>(l) >= static_cast<int>(level_.load()); }
  void log(LogLevel l, const std::string& logger, const std::string& msg, const Json& kv = Json());

 private:
  std::atomic<LogLevel> level_{LogLevel::Info};
  std::atomic<bool> json_{false};
  std::mutex mu_;
  std::function<void(const std::string&)> sink_;
};

#define KF_LOG(level, logger, msg, ...) \
  do { \
    if (::kf::Logger::get().enabled(level)) ::kf::Logger::get().log(level, logger, msg, ##__VA_ARGS__); \
  } while (0)
#define KF_INFO(logger, msg, ...) KF_LOG(::kf::LogLevel::Info, logger, msg, ##__VA_ARGS__)
#define KF_WARN(logger, msg, ...) KF_LOG(::kf::LogLevel::Warn, logger, msg, ##__VA_ARGS__)
#define KF_ERROR(logger, msg, ...) KF_LOG(::kf::LogLevel::Error, logger, msg, ##__VA_ARGS__)
#define KF_DEBUG(logger, msg, ...) KF_LOG(::kf::LogLevel::Debug, logger, msg, ##__VA_ARGS__)

// ---- flags ----------------------------------------------------------------------------------
// Go-flag-compatible parser: -name=value, --name=value, -name value, bool flags without value.
class Flags {
 public:
  void add_string(const std::string& name, std::string* dst, const std::string& def, const std::string& help);
  void add_int(const std::string& name, int64_t* dst, int64_t def, const std::string& help);
  void add_double(const std::string& name, double* dst, double def, const std::string& help);
  void add_bool(const std::string& name, bool* dst, bool def, const std::string& help);
  // returns false (and fills err) on unknown flag / bad value; "-h" sets help_requested.
  bool parse(int argc, char** argv, std::string* err);
  std::string usage() const;
  bool help_requested() const { return help_; }
  const std::vector<std::string>& positional() const { return pos_; }

 private:
  struct F {
    std::string kind, help, def;
    std::string* s = nullptr;
    int64_t* i = nullptr;
    double* d = nullptr;
    bool* b = nullptr;
  };
  std::map<std::string, F> flags_;
  std::vector<std::string> pos_;
  bool help_ = false;
};

}  // namespace kf
