// util.cc — see util.h.
#include <sys/random.h>
#include <cerrno>
#include <pthread.h>
#include "core/util.h"

#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <sstream>

namespace kf {

std::vector<std::string> split(const std::string& s, char sep, bool skip_empty) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      if (!(skip_empty && cur.empty())) out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!(skip_empty && cur.empty())) out.push_back(cur);
  return out;
}

std::string join(const std::vector<std::string>& parts, const std::string& sep) {
  std::string out;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) out += sep;
    out += parts[i];
  }
  return out;
}

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}
bool contains(const std::string& s, const std::string& p) { return s.find(p) != std::string::npos; }
std::string to_lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}
std::string to_upper(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
  return s;
}
std::string replace_all(std::string s, const std::string& from, const std::string& to) {
  if (from.empty()) return s;
  size_t pos = 0;
  while ((pos = s.find(from, pos)) != std::string::npos) {
    s.replace(pos, from.size(), to);
    pos += to.size();
  }
  return s;
}

std::string url_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      out += ' ';
    } else if (s[i] == '%' && i + 2 < s.size()) {
      out += static_cast<char>(std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else {
      out += s[i];
    }
  }
  return out;
}

std::string url_decode_path(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit(static_cast<unsigned char>(s[i + 1])) &&
        std::isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      out += static_cast<char>(std::strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else {
      out += s[i];  // '+' is a plus sign in a path (form encoding applies to queries only)
    }
  }
  return out;
}

bool path_has_escaped_slash(const std::string& raw_path) {
  const std::string l = to_lower(raw_path);
  return l.find("%2f") != std::string::npos || l.find("%5c") != std::string::npos;
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out += static_cast<char>(c);
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
  return out;
}

std::string base64_encode(const std::string& in) {
  static const char* t = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  size_t i = 0;
  while (i + 2 < in.size()) {
    uint32_t v = (uint8_t(in[i]) << 16) | (uint8_t(in[i + 1]) << 8) | uint8_t(in[i + 2]);
    out += t[v >> 18];
    out += t[(v >> 12) & 63];
    out += t[(v >> 6) & 63];
    out += t[v & 63];
    i += 3;
  }
  if (i + 1 == in.size()) {
    uint32_t v = uint8_t(in[i]) << 16;
    out += t[v >> 18];
    out += t[(v >> 12) & 63];
    out += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = (uint8_t(in[i]) << 16) | (uint8_t(in[i + 1]) << 8);
    out += t[v >> 18];
    out += t[(v >> 12) & 63];
    out += t[(v >> 6) & 63];
    out += '=';
  }
  return out;
}

std::string base64_decode(const std::string& in) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  std::string out;
  uint32_t buf = 0;
  int bits = 0;
  for (char c : in) {
    int v = val(c);
    if (v < 0) continue;
    buf = (buf << 6) | static_cast<uint32_t>(v);
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out += static_cast<char>((buf >> bits) & 0xFF);
    }
  }
  return out;
}

namespace {
std::mt19937_64& rng() {
  thread_local std::mt19937_64 r(std::random_device{}() ^ static_cast<uint64_t>(now_unix_ms()) ^
                                  reinterpret_cast<uintptr_t>(&r));
  return r;
}
}  // namespace

std::string random_hex(size_t nbytes) {
  static const char* hex = "0123456789abcdef";
  std::string out;
  for (size_t i = 0; i < nbytes; ++i) {
    unsigned v = static_cast<unsigned>(rng()() & 0xFF);
    out += hex[v >> 4];
    out += hex[v & 15];
  }
  return out;
}

std::string secure_random_hex(size_t nbytes) {
  static const char* hex = "0123456789abcdef";
  std::string raw(nbytes, '\0');
  size_t got = 0;
  while (got < nbytes) {
    const ssize_t n = ::getrandom(raw.data() + got, nbytes - got, 0);
    if (n < 0) {
      if (errno == EINTR) continue;
      std::abort();  // no entropy source: never hand out a predictable credential
    }
    got += static_cast<size_t>(n);
  }
  std::string out;
  for (unsigned char v : raw) {
    out += hex[v >> 4];
    out += hex[v & 15];
  }
  return out;
}

std::string random_alnum(size_t n) {
  static const char* chars = "bcdfghjklmnpqrstvwxz2456789";  // k8s generateName alphabet
  std::string out;
  for (size_t i = 0; i < n; ++i) out += chars[rng()() % 27];
  return out;
}

std::string uuid4() {
  std::string h = random_hex(16);
  h[12] = '4';
  h[16] = "89ab"[rng()() % 4];
  return h.substr(0, 8) + "-" + h.substr(8, 4) + "-" + h.substr(12, 4) + "-" + h.substr(16, 4) + "-" + h.substr(20, 12);
}

// resource.Quantity's grammar: <sign><digits>[.<digits>]<suffix>, suffix one of the binary SI
// (Ki..Ei), decimal SI (n u m "" k M G T P E) or a decimal exponent (e3, E-2). Anything else
// ("two", "1 Gi", "inf", "0x10", "1.2.3") is not a quantity.
std::optional<double> parse_quantity(const std::string& qin) {
  const std::string q = trim(qin);
  size_t i = 0;
  if (i < q.size() && (q[i] == '+' || q[i] == '-')) ++i;
  int digits = 0, dots = 0;
  for (; i < q.size() && (std::isdigit(static_cast<unsigned char>(q[i])) || q[i] == '.'); ++i) (q[i] == '.' ? dots : digits)++;
  if (digits == 0 || dots > 1) return std::nullopt;
  const std::string num = q.substr(0, i), suffix = q.substr(i);
  static const std::map<std::string, double> suffixes = {
      {"", 1.0}, {"Ki", 1024.0}, {"Mi", 1048576.0}, {"Gi", 1073741824.0}, {"Ti", 1099511627776.0},
      {"Pi", 1125899906842624.0}, {"Ei", 1152921504606846976.0},
      {"n", 1e-9}, {"u", 1e-6}, {"m", 1e-3}, {"k", 1e3}, {"M", 1e6}, {"G", 1e9}, {"T", 1e12},
      {"P", 1e15}, {"E", 1e18}};
  double mult = 1.0;
  auto it = suffixes.find(suffix);
  if (it != suffixes.end()) {
    mult = it->second;
  } else if (suffix[0] == 'e' || suffix[0] == 'E') {
    size_t j = 1;
    if (j < suffix.size() && (suffix[j] == '+' || suffix[j] == '-')) ++j;
    if (j == suffix.size() || suffix.find_first_not_of("0123456789", j) != std::string::npos) return std::nullopt;
    mult = std::pow(10.0, std::atof(suffix.c_str() + 1));
  } else {
    return std::nullopt;
  }
  return std::strtod(num.c_str(), nullptr) * mult;
}

std::string format_quantity_int(int64_t v) { return std::to_string(v); }

int64_t now_unix_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}
double now_seconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string rfc3339_from_ms(int64_t ms, bool with_ms) {
  time_t secs = static_cast<time_t>(ms / 1000);
  struct tm tm_utc;
  gmtime_r(&secs, &tm_utc);
  char buf[64];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm_utc);
  std::string out = buf;
  if (with_ms) {
    char frac[8];
    std::snprintf(frac, sizeof frac, ".%03d", static_cast<int>(ms % 1000));
    out += frac;
  }
  out += "Z";
  return out;
}
std::string rfc3339_now() { return rfc3339_from_ms(now_unix_ms(), false); }
std::string rfc3339_ms_now() { return rfc3339_from_ms(now_unix_ms(), true); }

std::optional<int64_t> parse_rfc3339_ms(const std::string& s) {
  int Y, M, D, h, m;
  double sec;
  if (s.size() < 20) return std::nullopt;
  if (std::sscanf(s.c_str(), "%d-%d-%dT%d:%d:%lf", &Y, &M, &D, &h, &m, &sec) != 6) return std::nullopt;
  struct tm tm_utc {};
  tm_utc.tm_year = Y - 1900;
  tm_utc.tm_mon = M - 1;
  tm_utc.tm_mday = D;
  tm_utc.tm_hour = h;
  tm_utc.tm_min = m;
  tm_utc.tm_sec = 0;
  time_t t = timegm(&tm_utc);
  int64_t ms = static_cast<int64_t>(t) * 1000 + static_cast<int64_t>(std::llround(sec * 1000.0));
  // timezone offset (+hh:mm / -hh:mm); 'Z' or nothing = UTC
  size_t tpos = s.find('T');
  size_t zpos = s.find_first_of("+-", tpos);
  if (zpos != std::string::npos && zpos > tpos) {
    int oh = 0, om = 0;
    if (std::sscanf(s.c_str() + zpos + 1, "%d:%d", &oh, &om) >= 1) {
      int64_t off = (oh * 60 + om) * 60000LL;
      ms += (s[zpos] == '+') ? -off : off;
    }
  }
  return ms;
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

bool write_file(const std::string& path, const std::string& data) {
  std::string tmp = path + ".tmp." + random_hex(4);
  {
    std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
    if (!f) return false;
    f << data;
    if (!f) return false;
  }
  return std::rename(tmp.c_str(), path.c_str()) == 0;
}

bool file_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

bool make_dirs(const std::string& path) {
  if (path.empty()) return false;
  std::string cur;
  for (const auto& part : split(path, '/')) {
    if (part.empty()) {
      if (cur.empty()) cur = "/";
      continue;
    }
    cur += (cur.empty() || cur.back() == '/') ? part : "/" + part;
    if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
  }
  return true;
}

int64_t file_mtime_ns(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return -1;
  return static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000LL + st.st_mtim.tv_nsec;
}

std::string getenv_or(const char* name, const std::string& def) {
  const char* v = std::getenv(name);
  return v ? std::string(v) : def;
}

bool env_true(const char* name, bool def) {
  const char* v = std::getenv(name);
  if (!v) return def;
  std::string s = to_lower(v);
  return s == "1" || s == "true" || s == "yes" || s == "on";
}

// ---- logging --------------------------------------------------------------------------------
Logger& Logger::get() {
  static Logger l;
  return l;
}
void Logger::set_sink(std::function<void(const std::string&)> sink) {
  std::lock_guard<std::mutex> g(mu_);
  sink_ = std::move(sink);
}
void Logger::log(LogLevel l, const std::string& logger, const std::string& msg, const Json& kv) {
  static const char* names[] = {"debug", "info", "warn", "error"};
  std::string line;
  if (json_) {
    Json j = Json::object();
    j["level"] = names[static_cast<int>(l)];
    j["ts"] = rfc3339_ms_now();
    j["logger"] = logger;
    j["msg"] = msg;
    for (const auto& m : kv.as_object()) j[m.first] = m.second;
    line = j.dump();
  } else {
    line = rfc3339_ms_now() + "\t" + names[static_cast<int>(l)] + "\t" + logger + "\t" + msg;
    if (kv.is_object() && !kv.empty()) line += "\t" + kv.dump();
  }
  std::lock_guard<std::mutex> g(mu_);
  if (sink_) {
    sink_(line);
  } else {
    std::fprintf(stderr, "%s\n", line.c_str());
  }
}

// ---- flags ----------------------------------------------------------------------------------
void Flags::add_string(const std::string& name, std::string* dst, const std::string& def, const std::string& help) {
  *dst = def;
  F f;
  f.kind = "string";
  f.help = help;
  f.def = def;
  f.s = dst;
  flags_[name] = f;
}
void Flags::add_int(const std::string& name, int64_t* dst, int64_t def, const std::string& help) {
  *dst = def;
  F f;
  f.kind = "int";
  f.help = help;
  f.def = std::to_string(def);
  f.i = dst;
  flags_[name] = f;
}
void Flags::add_double(const std::string& name, double* dst, double def, const std::string& help) {
  *dst = def;
  F f;
  f.kind = "float";
  f.help = help;
  f.def = std::to_string(def);
  f.d = dst;
  flags_[name] = f;
}
void Flags::add_bool(const std::string& name, bool* dst, bool def, const std::string& help) {
  *dst = def;
  F f;
  f.kind = "bool";
  f.help = help;
  f.def = def ? "true" : "false";
  f.b = dst;
  flags_[name] = f;
}
bool Flags::parse(int argc, char** argv, std::string* err) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-h" || a == "--help" || a == "-help") {
      help_ = true;
      continue;
    }
    if (a.size() < 2 || a[0] != '-') {
      pos_.push_back(a);
      continue;
    }
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    std::string name = body, value;
    bool has_value = false;
    size_t eq = body.find('=');
    if (eq != std::string::npos) {
      name = body.substr(0, eq);
      value = body.substr(eq + 1);
      has_value = true;
    }
    auto it = flags_.find(name);
    if (it == flags_.end()) {
      // zap-style flags (--zap-log-level=...) are accepted and ignored for compatibility
      if (starts_with(name, "zap-") || starts_with(name, "kubeconfig")) {
        if (!has_value && i + 1 < argc && argv[i + 1][0] != '-') ++i;
        continue;
      }
      if (err) *err = "unknown flag: -" + name;
      return false;
    }
    F& f = it->second;
    if (f.kind == "bool") {
      if (!has_value) value = "true";
      std::string v = to_lower(value);
      *f.b = (v == "true" || v == "1" || v == "yes");
      continue;
    }
    if (!has_value) {
      if (i + 1 >= argc) {
        if (err) *err = "flag needs an argument: -" + name;
        return false;
      }
      value = argv[++i];
    }
    if (f.kind == "string") {
      *f.s = value;
    } else if (f.kind == "int") {
      char* end = nullptr;
      *f.i = std::strtoll(value.c_str(), &end, 10);
      if (!end || *end) {
        if (err) *err = "invalid int for -" + name + ": " + value;
        return false;
      }
    } else if (f.kind == "float") {
      char* end = nullptr;
      *f.d = std::strtod(value.c_str(), &end);
      if (!end || *end) {
        if (err) *err = "invalid float for -" + name + ": " + value;
        return false;
      }
    }
  }
  return true;
}
std::string Flags::usage() const {
  std::string out = "Flags:\n";
  for (const auto& kv : flags_)
    out += "  -" + kv.first + " (" + kv.second.kind + ", default \"" + kv.second.def + "\")\n      " + kv.second.help + "\n";
  return out;
}

void set_thread_name(const std::string& name) {
  const std::string n = name.substr(0, 15);
  ::pthread_setname_np(::pthread_self(), n.c_str());
}

}  // namespace kf
