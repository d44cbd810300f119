// http.cc — see http.h.
#include "core/http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

#include "core/util.h"

namespace kf {

bool CaseLess::operator()(const std::string& a, const std::string& b) const {
  return std::lexicographical_compare(a.begin(), a.end(), b.begin(), b.end(), [](char x, char y) {
    return std::tolower(static_cast<unsigned char>(x)) < std::tolower(static_cast<unsigned char>(y));
  });
}

std::string HttpRequest::header(const std::string& name, const std::string& def) const {
  auto it = headers.find(name);
  return it == headers.end() ? def : it->second;
}
std::string HttpRequest::q(const std::string& name, const std::string& def) const {
  auto it = query.find(name);
  return (it == query.end() || it->second.empty()) ? def : it->second.front();
}
std::string HttpRequest::param(const std::string& name) const {
  auto it = params.find(name);
  return it == params.end() ? "" : it->second;
}

const char* http_status_text(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 304: return "Not Modified";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Status";
  }
}

// ---- router -----------------------------------------------------------------------------------
void Router::add(const std::string& method, const std::string& pattern, Handler h) {
  Route r;
  r.method = method;
  std::string p = pattern;
  if (ends_with(p, "/*")) {
    r.prefix = true;
    p = p.substr(0, p.size() - 2);
  }
  r.segs = split(p, '/', true);
  r.h = std::move(h);
  routes_.push_back(std::move(r));
}

void Router::dispatch(HttpRequest& req, HttpResponse& resp) const {
  auto segs = split(req.path, '/', true);
  bool method_mismatch = false;
  for (const auto& r : routes_) {
    if (!r.prefix && r.segs.size() != segs.size()) continue;
    if (r.prefix && segs.size() < r.segs.size()) continue;
    std::map<std::string, std::string> params;
    bool ok = true;
    for (size_t i = 0; i < r.segs.size() && ok; ++i) {
      const std::string& ps = r.segs[i];
      if (ps.size() > 2 && ps.front() == '{' && ps.back() == '}') {
        params[ps.substr(1, ps.size() - 2)] = url_decode(segs[i]);
      } else if (ps != segs[i]) {
        ok = false;
      }
    }
    if (!ok) continue;
    if (r.method != "*" && r.method != req.method) {
      method_mismatch = true;
      continue;
    }
    req.params = std::move(params);
    r.h(req, resp);
    return;
  }
  if (method_mismatch) {
    resp.json(405, R"({"error":"method not allowed"})");
    return;
  }
  if (not_found_) {
    not_found_(req, resp);
  } else {
    resp.json(404, R"({"error":"not found"})");
  }
}

// ---- connections (plain TCP or TLS) -------------------------------------------------------------
namespace {

std::string tls_error(const std::string& what) {
  std::string out = what;
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    char buf[256];
    ERR_error_string_n(e, buf, sizeof buf);
    out += std::string(": ") + buf;
  }
  return out;
}

class Conn : public RawConn {
 public:
  Conn(int fd, SSL* ssl, bool own_fd) : fd_(fd), ssl_(ssl), own_fd_(own_fd) {}
  using RawConn::write;
  ~Conn() override {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
    }
    if (own_fd_ && fd_ >= 0) ::close(fd_);
  }
  long read(char* buf, size_t n) override {
    for (;;) {
      if (!ssl_) {
        ssize_t r = ::recv(fd_, buf, n, 0);
        if (r < 0 && errno == EINTR) continue;
        return static_cast<long>(r);
      }
      ERR_clear_error();
      errno = 0;
      int r = SSL_read(ssl_, buf, static_cast<int>(std::min<size_t>(n, 1 << 30)));
      if (r > 0) return r;
      int e = SSL_get_error(ssl_, r);
      if (e == SSL_ERROR_ZERO_RETURN) return 0;
      if (e == SSL_ERROR_SYSCALL && errno == EINTR) continue;
      if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) {
        errno = EAGAIN;  // receive timeout on the blocking socket
        return -1;
      }
      if (e == SSL_ERROR_SYSCALL && errno == 0) return 0;  // peer closed without close_notify
      return -1;
    }
  }
  bool write(const char* p, size_t n) override {
    while (n > 0) {
      if (!ssl_) {
        ssize_t w = ::send(fd_, p, n, MSG_NOSIGNAL);
        if (w < 0) {
          if (errno == EINTR) continue;
          return false;
        }
        p += w;
        n -= static_cast<size_t>(w);
        continue;
      }
      ERR_clear_error();
      int w = SSL_write(ssl_, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
      if (w <= 0) {
        int e = SSL_get_error(ssl_, w);
        if (e == SSL_ERROR_SYSCALL && errno == EINTR) continue;
        return false;
      }
      p += w;
      n -= static_cast<size_t>(w);
    }
    return true;
  }
  int fd() const override { return fd_; }
  bool has_buffered() const override { return ssl_ && SSL_pending(ssl_) > 0; }
  void set_timeout_ms(int ms) override {
    struct timeval tv;
    tv.tv_sec = ms / 1000;
    tv.tv_usec = (ms % 1000) * 1000;
    ::setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    ::setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  }

 private:
  int fd_;
  SSL* ssl_;
  bool own_fd_;
};

// Buffered reader over a connection.
class Reader {
 public:
  explicit Reader(RawConn& c) : c_(c) {}
  // returns false on EOF/error/timeout
  bool fill() {
    char tmp[16384];
    long r = c_.read(tmp, sizeof tmp);
    if (r > 0) {
      buf_.append(tmp, static_cast<size_t>(r));
      return true;
    }
    last_timeout_ = r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK);
    return false;
  }
  bool read_line(std::string& line, size_t max = 1 << 20) {
    for (;;) {
      size_t p = buf_.find('\n', pos_);
      if (p != std::string::npos) {
        line.assign(buf_, pos_, p - pos_);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos_ = p + 1;
        compact();
        return true;
      }
      if (buf_.size() - pos_ > max) return false;
      if (!fill()) return false;
    }
  }
  bool read_n(std::string& out, size_t n) {
    while (buf_.size() - pos_ < n)
      if (!fill()) return false;
    out.append(buf_, pos_, n);
    pos_ += n;
    compact();
    return true;
  }
  bool read_to_eof(std::string& out) {
    out.append(buf_, pos_, std::string::npos);
    buf_.clear();
    pos_ = 0;
    char tmp[16384];
    for (;;) {
      long r = c_.read(tmp, sizeof tmp);
      if (r > 0) {
        out.append(tmp, static_cast<size_t>(r));
        continue;
      }
      return r == 0;
    }
  }
  // up to max buffered bytes (reading once from the connection when none are buffered)
  int read_some(std::string& out, size_t max) {
    if (buf_.size() == pos_) {
      buf_.clear();
      pos_ = 0;
      if (!fill()) return last_timeout_ ? -2 : 0;
    }
    size_t take = std::min(max, buf_.size() - pos_);
    out.append(buf_, pos_, take);
    pos_ += take;
    compact();
    return static_cast<int>(take);
  }
  std::string take_buffered() {
    std::string out = buf_.substr(pos_);
    buf_.clear();
    pos_ = 0;
    return out;
  }
  size_t buffered() const { return buf_.size() - pos_; }
  bool last_timeout() const { return last_timeout_; }

 private:
  void compact() {
    if (pos_ > 65536) {
      buf_.erase(0, pos_);
      pos_ = 0;
    }
  }
  RawConn& c_;
  std::string buf_;
  size_t pos_ = 0;
  bool last_timeout_ = false;
};

bool read_headers(Reader& rd, Headers& h) {
  std::string line;
  for (;;) {
    if (!rd.read_line(line)) return false;
    if (line.empty()) return true;
    size_t c = line.find(':');
    if (c == std::string::npos) continue;
    h[trim(line.substr(0, c))] = trim(line.substr(c + 1));
  }
}

bool read_body(Reader& rd, const Headers& h, std::string& body, bool until_eof) {
  auto te = h.find("Transfer-Encoding");
  if (te != h.end() && contains(to_lower(te->second), "chunked")) {
    std::string line;
    for (;;) {
      if (!rd.read_line(line)) return false;
      size_t n = std::strtoul(line.c_str(), nullptr, 16);
      if (n == 0) {
        rd.read_line(line);  // trailing CRLF
        return true;
      }
      if (!rd.read_n(body, n)) return false;
      if (!rd.read_line(line)) return false;
    }
  }
  auto cl = h.find("Content-Length");
  if (cl != h.end()) {
    size_t n = std::strtoul(cl->second.c_str(), nullptr, 10);
    if (n > (512u << 20)) return false;
    return rd.read_n(body, n);
  }
  if (until_eof) return rd.read_to_eof(body);
  return true;
}

void parse_query(const std::string& raw, std::map<std::string, std::vector<std::string>>& out) {
  for (const auto& kv : split(raw, '&', true)) {
    size_t e = kv.find('=');
    if (e == std::string::npos) out[url_decode(kv)].push_back("");
    else out[url_decode(kv.substr(0, e))].push_back(url_decode(kv.substr(e + 1)));
  }
}

class ChunkWriter : public StreamWriter {
 public:
  explicit ChunkWriter(RawConn& c) : c_(c) {}
  bool write(const std::string& data) override {
    if (dead_) return false;
    if (data.empty()) return true;
    char hdr[32];
    std::snprintf(hdr, sizeof hdr, "%zx\r\n", data.size());
    if (!c_.write(std::string(hdr) + data + "\r\n")) dead_ = true;
    return !dead_;
  }
  bool alive() override {
    if (dead_) return false;
    struct pollfd p {c_.fd(), POLLIN | POLLRDHUP, 0};
    int r = ::poll(&p, 1, 0);
    if (r > 0 && (p.revents & (POLLHUP | POLLERR | POLLRDHUP))) dead_ = true;
    if (r > 0 && (p.revents & POLLIN)) {
      char c;
      ssize_t n = ::recv(c_.fd(), &c, 1, MSG_PEEK | MSG_DONTWAIT);
      if (n == 0) dead_ = true;
    }
    return !dead_;
  }
  bool finish() { return !dead_ && c_.write("0\r\n\r\n"); }

 private:
  RawConn& c_;
  bool dead_ = false;
};

HostResolver& resolver_slot() {
  static HostResolver r;
  return r;
}
std::mutex& resolver_mu() {
  static std::mutex m;
  return m;
}

int connect_to(const std::string& host_in, int port_in, int timeout_ms, std::string* err) {
  std::string host = host_in;
  int port = port_in;
  {
    HostResolver r;
    {
      std::lock_guard<std::mutex> g(resolver_mu());
      r = resolver_slot();
    }
    std::string ip;
    int p2 = port;
    if (r && r(host_in, port_in, ip, p2)) {
      host = ip;
      port = p2;
    }
  }
  struct addrinfo hints {};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  struct addrinfo* res = nullptr;
  std::string ps = std::to_string(port);
  int gai = ::getaddrinfo(host.c_str(), ps.c_str(), &hints, &res);
  if (gai != 0 || !res) {
    if (err) *err = "resolve " + host + ": " + gai_strerror(gai);
    return -1;
  }
  int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    ::freeaddrinfo(res);
    if (err) *err = "socket failed";
    return -1;
  }
  int fl = ::fcntl(fd, F_GETFL, 0);
  ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0 && errno != EINPROGRESS) {
    if (err) *err = std::string("connect: ") + std::strerror(errno);
    ::close(fd);
    return -1;
  }
  if (rc != 0) {
    struct pollfd p {fd, POLLOUT, 0};
    int pr = ::poll(&p, 1, timeout_ms);
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
    if (pr <= 0 || soerr != 0) {
      if (err) *err = pr <= 0 ? "connect timeout" : std::string("connect: ") + std::strerror(soerr);
      ::close(fd);
      return -1;
    }
  }
  ::fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  return fd;
}

void set_timeouts(int fd, int ms) {
  struct timeval tv;
  tv.tv_sec = ms / 1000;
  tv.tv_usec = (ms % 1000) * 1000;
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}


std::shared_ptr<SSL_CTX> make_server_ctx(const TlsServerConfig& c, std::string* err) {
  std::shared_ptr<SSL_CTX> ctx(SSL_CTX_new(TLS_server_method()), SSL_CTX_free);
  if (!ctx) {
    if (err) *err = tls_error("SSL_CTX_new");
    return nullptr;
  }
  SSL_CTX_set_min_proto_version(ctx.get(), TLS1_2_VERSION);
  if (SSL_CTX_use_certificate_chain_file(ctx.get(), c.cert_file.c_str()) != 1) {
    if (err) *err = tls_error("load certificate " + c.cert_file);
    return nullptr;
  }
  if (SSL_CTX_use_PrivateKey_file(ctx.get(), c.key_file.c_str(), SSL_FILETYPE_PEM) != 1 ||
      SSL_CTX_check_private_key(ctx.get()) != 1) {
    if (err) *err = tls_error("load private key " + c.key_file);
    return nullptr;
  }
  if (!c.client_ca_file.empty()) {
    if (SSL_CTX_load_verify_locations(ctx.get(), c.client_ca_file.c_str(), nullptr) != 1) {
      if (err) *err = tls_error("load client CA " + c.client_ca_file);
      return nullptr;
    }
    SSL_CTX_set_verify(ctx.get(), SSL_VERIFY_PEER | (c.require_client_cert ? SSL_VERIFY_FAIL_IF_NO_PEER_CERT : 0), nullptr);
  }
  return ctx;
}

// client contexts, cached per option set (loading a CA bundle costs milliseconds)
std::mutex& tls_client_mu() {
  static std::mutex m;
  return m;
}
TlsClientOptions& tls_client_default() {
  static TlsClientOptions o;
  return o;
}
std::shared_ptr<SSL_CTX> build_client_ctx(const TlsClientOptions& o, std::string* err);

// A file's identity for the cache key: a rotated service-account ca.crt or client certificate (same
// path, new content) must build a fresh context, so mtime + size are part of the key.
std::string file_stamp(const std::string& path) {
  struct stat st {};
  if (path.empty() || ::stat(path.c_str(), &st) != 0) return "-";
  return std::to_string((long long)st.st_mtim.tv_sec) + "." + std::to_string((long long)st.st_mtim.tv_nsec) + ":" +
         std::to_string((long long)st.st_size);
}

std::shared_ptr<SSL_CTX> client_ctx(const TlsClientOptions& o, std::string* err) {
  // keyed by the option set plus the files' current stamps; superseded entries (a rotated file, or
  // a webhook caBundle that changed) are evicted so the cache cannot grow without bound
  static std::map<std::string, std::pair<std::string, std::shared_ptr<SSL_CTX>>> cache;  // opts -> (stamps, ctx)
  const std::string key = o.ca_file + '\0' + o.ca_pem + '\0' + o.cert_file + '\0' + o.key_file + '\0' +
                          (o.insecure_skip_verify ? "1" : "0");
  const std::string stamps = file_stamp(o.ca_file) + '|' + file_stamp(o.cert_file) + '|' + file_stamp(o.key_file);
  std::lock_guard<std::mutex> g(tls_client_mu());
  auto it = cache.find(key);
  if (it != cache.end() && it->second.first == stamps) return it->second.second;
  if (it != cache.end()) cache.erase(it);
  if (cache.size() >= 64) cache.clear();  // bounded: caBundle-keyed entries of deleted webhooks
  auto made = build_client_ctx(o, err);
  if (made) cache[key] = {stamps, made};
  return made;
}

std::shared_ptr<SSL_CTX> build_client_ctx(const TlsClientOptions& o, std::string* err) {
  std::shared_ptr<SSL_CTX> ctx(SSL_CTX_new(TLS_client_method()), SSL_CTX_free);
  if (!ctx) {
    if (err) *err = tls_error("SSL_CTX_new");
    return nullptr;
  }
  SSL_CTX_set_min_proto_version(ctx.get(), TLS1_2_VERSION);
  if (o.insecure_skip_verify) {
    SSL_CTX_set_verify(ctx.get(), SSL_VERIFY_NONE, nullptr);
  } else {
    SSL_CTX_set_verify(ctx.get(), SSL_VERIFY_PEER, nullptr);
    bool loaded = false;
    if (!o.ca_file.empty()) {
      if (SSL_CTX_load_verify_locations(ctx.get(), o.ca_file.c_str(), nullptr) != 1) {
        if (err) *err = tls_error("load CA bundle " + o.ca_file);
        return nullptr;
      }
      loaded = true;
    }
    if (!o.ca_pem.empty()) {
      std::unique_ptr<BIO, decltype(&BIO_free)> bio(BIO_new_mem_buf(o.ca_pem.data(), static_cast<int>(o.ca_pem.size())),
                                                    BIO_free);
      X509_STORE* store = SSL_CTX_get_cert_store(ctx.get());
      int n = 0;
      while (X509* x = PEM_read_bio_X509(bio.get(), nullptr, nullptr, nullptr)) {
        X509_STORE_add_cert(store, x);
        X509_free(x);
        ++n;
      }
      ERR_clear_error();  // the read loop ends on a "no start line" error
      if (n == 0) {
        if (err) *err = "CA bundle holds no PEM certificate";
        return nullptr;
      }
      loaded = true;
    }
    if (!loaded) SSL_CTX_set_default_verify_paths(ctx.get());
  }
  if (!o.cert_file.empty()) {
    if (SSL_CTX_use_certificate_chain_file(ctx.get(), o.cert_file.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx.get(), (o.key_file.empty() ? o.cert_file : o.key_file).c_str(), SSL_FILETYPE_PEM) != 1) {
      if (err) *err = tls_error("load client certificate " + o.cert_file);
      return nullptr;
    }
  }
  return ctx;
}

bool is_ip_literal(const std::string& host) {
  struct in_addr a4;
  struct in6_addr a6;
  return ::inet_pton(AF_INET, host.c_str(), &a4) == 1 || ::inet_pton(AF_INET6, host.c_str(), &a6) == 1;
}

// connect + (https) handshake with hostname verification against the URL's host
std::unique_ptr<Conn> open_conn(const Url& u, int timeout_ms, std::string* err, const TlsClientOptions* tls) {
  if (u.scheme != "http" && u.scheme != "https") {
    if (err) *err = "unsupported scheme " + u.scheme;
    return nullptr;
  }
  int fd = connect_to(u.host, u.port, timeout_ms, err);
  if (fd < 0) return nullptr;
  set_timeouts(fd, timeout_ms);
  if (u.scheme == "http") return std::make_unique<Conn>(fd, nullptr, true);
  TlsClientOptions opts = tls ? *tls : default_tls_client();
  auto ctx = client_ctx(opts, err);
  if (!ctx) {
    ::close(fd);
    return nullptr;
  }
  SSL* ssl = SSL_new(ctx.get());
  SSL_set_fd(ssl, fd);
  if (!is_ip_literal(u.host)) SSL_set_tlsext_host_name(ssl, u.host.c_str());
  if (!opts.insecure_skip_verify) {
    X509_VERIFY_PARAM* vp = SSL_get0_param(ssl);
    if (is_ip_literal(u.host)) X509_VERIFY_PARAM_set1_ip_asc(vp, u.host.c_str());
    else X509_VERIFY_PARAM_set1_host(vp, u.host.c_str(), 0);
  }
  ERR_clear_error();
  if (SSL_connect(ssl) != 1) {
    long vr = SSL_get_verify_result(ssl);
    if (err) {
      *err = vr != X509_V_OK ? std::string("tls: certificate verify failed: ") + X509_verify_cert_error_string(vr)
                             : tls_error("tls handshake with " + u.host);
    }
    SSL_free(ssl);
    ::close(fd);
    return nullptr;
  }
  return std::make_unique<Conn>(fd, ssl, true);
}

}  // namespace

void set_default_tls_client(const TlsClientOptions& o) {
  std::lock_guard<std::mutex> g(tls_client_mu());
  tls_client_default() = o;
}
TlsClientOptions default_tls_client() {
  std::lock_guard<std::mutex> g(tls_client_mu());
  return tls_client_default();
}

// ---- server ------------------------------------------------------------------------------------
HttpServer::HttpServer() { ::signal(SIGPIPE, SIG_IGN); }
HttpServer::~HttpServer() { stop(); }

bool HttpServer::enable_tls(const TlsServerConfig& cfg, std::string* err) {
  auto ctx = make_server_ctx(cfg, err);
  if (!ctx) return false;
  std::lock_guard<std::mutex> g(tls_mu_);
  tls_cfg_ = cfg;
  tls_ctx_ = ctx;
  tls_mtime_ = file_mtime_ns(cfg.cert_file) ^ (file_mtime_ns(cfg.key_file) << 1);
  tls_checked_ = now_seconds();
  return true;
}

std::shared_ptr<SSL_CTX> HttpServer::current_tls_ctx() {
  std::lock_guard<std::mutex> g(tls_mu_);
  if (!tls_ctx_) return nullptr;
  const double now = now_seconds();
  if (now - tls_checked_ >= 0.2) {  // certwatcher: a rotated pair is served from the next connection on
    tls_checked_ = now;
    const long long m = file_mtime_ns(tls_cfg_.cert_file) ^ (file_mtime_ns(tls_cfg_.key_file) << 1);
    if (m != tls_mtime_) {
      std::string err;
      auto ctx = make_server_ctx(tls_cfg_, &err);
      if (ctx) {
        tls_ctx_ = ctx;
        tls_mtime_ = m;
        KF_INFO("http", "reloaded TLS certificate", Json{{"cert", tls_cfg_.cert_file}});
      } else {
        // a half-written pair: keep serving the old one, retry on a later connection
        KF_WARN("http", "TLS certificate reload failed", Json{{"error", err}});
      }
    }
  }
  return tls_ctx_;
}

bool HttpServer::listen(const std::string& addr, int port, std::string* err) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    if (err) *err = "socket failed";
    return false;
  }
  int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  struct sockaddr_in sa {};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  std::string a = addr.empty() ? "0.0.0.0" : addr;
  if (::inet_pton(AF_INET, a.c_str(), &sa.sin_addr) != 1) {
    if (err) *err = "bad listen address " + a;
    ::close(fd);
    return false;
  }
  if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    if (err) *err = "bind " + a + ":" + std::to_string(port) + ": " + std::strerror(errno);
    ::close(fd);
    return false;
  }
  if (::listen(fd, 512) != 0) {
    if (err) *err = std::string("listen: ") + std::strerror(errno);
    ::close(fd);
    return false;
  }
  socklen_t sl = sizeof sa;
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &sl);
  port_ = ntohs(sa.sin_port);
  addr_ = a;
  listen_fd_ = fd;
  return true;
}

void HttpServer::start() {
  running_ = true;
  const int fd = listen_fd_;
  accept_thread_ = std::thread([this, fd] { accept_loop(fd); });
}

void HttpServer::stop() {
  if (!running_.exchange(false)) return;
  // shutdown() wakes the accept thread; the fd is closed only after it has exited, so its number
  // cannot be reused by another socket while the loop still polls it (found by TSAN)
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (accept_thread_.joinable()) accept_thread_.join();
  if (listen_fd_ >= 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (int fd : conn_fds_) ::shutdown(fd, SHUT_RDWR);
  }
  // wait (bounded) for connection threads to observe the shutdown
  for (int i = 0; i < 500 && active_.load() > 0; ++i) ::usleep(10000);
}

void HttpServer::accept_loop(int listen_fd) {
  while (running_) {
    struct pollfd p {listen_fd, POLLIN, 0};
    int pr = ::poll(&p, 1, 200);
    if (pr <= 0) continue;
    struct sockaddr_in ca {};
    socklen_t cl = sizeof ca;
    int fd = ::accept4(listen_fd, reinterpret_cast<sockaddr*>(&ca), &cl, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    char ip[64];
    ::inet_ntop(AF_INET, &ca.sin_addr, ip, sizeof ip);
    std::string remote = std::string(ip) + ":" + std::to_string(ntohs(ca.sin_port));
    {
      std::lock_guard<std::mutex> g(conns_mu_);
      conn_fds_.push_back(fd);
    }
    active_++;
    std::thread([this, fd, remote] {
      set_thread_name("http-conn");
      serve_conn(fd, remote);
      {
        std::lock_guard<std::mutex> g(conns_mu_);
        conn_fds_.erase(std::remove(conn_fds_.begin(), conn_fds_.end(), fd), conn_fds_.end());
      }
      ::close(fd);
      active_--;
    }).detach();
  }
}

void HttpServer::serve_conn(int fd, std::string remote) {
  set_timeouts(fd, 120000);
  SSL* ssl = nullptr;
  if (auto ctx = current_tls_ctx()) {
    set_timeouts(fd, 10000);  // handshake budget
    ssl = SSL_new(ctx.get());
    SSL_set_fd(ssl, fd);
    ERR_clear_error();
    if (SSL_accept(ssl) != 1) {
      KF_DEBUG("http", "TLS handshake failed", Json{{"remote", remote}, {"error", tls_error("SSL_accept")}});
      SSL_free(ssl);
      return;
    }
    set_timeouts(fd, 120000);
  }
  Conn conn(fd, ssl, false);  // the accept thread's wrapper closes fd
  Reader rd(conn);
  while (running_) {
    HttpRequest req;
    std::string line;
    if (!rd.read_line(line)) return;
    if (line.empty()) continue;
    auto parts = split(line, ' ', true);
    if (parts.size() < 3) return;
    req.method = parts[0];
    req.target = parts[1];
    std::string version = parts[2];
    if (!read_headers(rd, req.headers)) return;
    if (!read_body(rd, req.headers, req.body, false)) return;
    size_t qm = req.target.find('?');
    req.path = url_decode_path(qm == std::string::npos ? req.target : req.target.substr(0, qm));
    if (qm != std::string::npos) {
      req.raw_query = req.target.substr(qm + 1);
      parse_query(req.raw_query, req.query);
    }
    req.remote_addr = remote;
    bool keep_alive = version == "HTTP/1.1" ? to_lower(req.header("Connection")) != "close"
                                            : to_lower(req.header("Connection")) == "keep-alive";
    HttpResponse resp;
    try {
      if (handler_) handler_(req, resp);
      else resp.json(404, R"({"error":"no handler"})");
    } catch (const std::exception& e) {
      resp = HttpResponse();
      resp.json(500, std::string(R"({"error":)") + json_quote(e.what()) + "}");
    }
    if (resp.upgrade) {
      const std::string pending = rd.take_buffered();
      conn.set_timeout_ms(0);  // a tunnel may idle for as long as its peers like
      resp.upgrade(conn, pending);
      return;
    }
    std::string head = "HTTP/1.1 " + std::to_string(resp.status) + " " + http_status_text(resp.status) + "\r\n";
    if (resp.stream) {
      for (const auto& h : resp.headers) head += h.first + ": " + h.second + "\r\n";
      head += "Transfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
      if (!conn.write(head)) return;
      ChunkWriter w(conn);
      resp.stream(w);
      w.finish();
      return;
    }
    if (!resp.headers.count("Content-Type")) resp.headers["Content-Type"] = "application/json";
    for (const auto& h : resp.headers) head += h.first + ": " + h.second + "\r\n";
    head += "Content-Length: " + std::to_string(resp.body.size()) + "\r\n";
    head += keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
    if (req.method != "HEAD") head += resp.body;  // one write: one TLS record for small responses
    if (!conn.write(head)) return;
    if (!keep_alive) return;
  }
}

// ---- client ------------------------------------------------------------------------------------
bool Url::parse(const std::string& url, Url& out) {
  std::string rest = url;
  size_t s = rest.find("://");
  if (s != std::string::npos) {
    out.scheme = to_lower(rest.substr(0, s));
    rest = rest.substr(s + 3);
  }
  size_t slash = rest.find('/');
  std::string hostport = slash == std::string::npos ? rest : rest.substr(0, slash);
  std::string pathq = slash == std::string::npos ? "/" : rest.substr(slash);
  size_t colon = hostport.rfind(':');
  out.port = out.scheme == "https" ? 443 : 80;
  if (colon != std::string::npos) {
    out.host = hostport.substr(0, colon);
    out.port = std::atoi(hostport.substr(colon + 1).c_str());
  } else {
    out.host = hostport;
  }
  size_t q = pathq.find('?');
  out.path = q == std::string::npos ? pathq : pathq.substr(0, q);
  out.query = q == std::string::npos ? "" : pathq.substr(q + 1);
  return !out.host.empty();
}

void set_host_resolver(HostResolver r) {
  std::lock_guard<std::mutex> g(resolver_mu());
  resolver_slot() = std::move(r);
}

namespace {
class ClientResponse : public HttpClientResponse {
 public:
  explicit ClientResponse(std::unique_ptr<Conn> c) : c_(std::move(c)), rd_(*c_) {}
  Reader& reader() { return rd_; }
  Next next(std::string& piece) override {
    if (done_) return kEnd;
    if (chunked) {
      if (chunk_left_ == 0) {
        std::string line;
        if (!rd_.read_line(line)) return rd_.last_timeout() ? kTimeout : kError;
        if (line.empty()) {  // CRLF that ended the previous chunk
          if (!rd_.read_line(line)) return rd_.last_timeout() ? kTimeout : kError;
        }
        chunk_left_ = std::strtoull(line.c_str(), nullptr, 16);
        if (chunk_left_ == 0) {
          rd_.read_line(line);  // trailer CRLF
          done_ = true;
          return kEnd;
        }
      }
      std::string out;
      int r = rd_.read_some(out, static_cast<size_t>(std::min<unsigned long long>(chunk_left_, 1 << 16)));
      if (r == -2) return kTimeout;
      if (r <= 0) return kError;
      chunk_left_ -= static_cast<unsigned long long>(r);
      piece = std::move(out);
      return kData;
    }
    if (length >= 0 && got_ >= length) {
      done_ = true;
      return kEnd;
    }
    std::string out;
    const size_t want = length >= 0 ? static_cast<size_t>(std::min<long long>(length - got_, 1 << 16)) : (1 << 16);
    int r = rd_.read_some(out, want);
    if (r == -2) return kTimeout;
    if (r == 0) {
      done_ = true;
      return length >= 0 ? kError : kEnd;  // EOF-delimited body ends here
    }
    if (r < 0) return kError;
    got_ += r;
    piece = std::move(out);
    return kData;
  }
  RawConn& conn() override { return *c_; }

 private:
  std::unique_ptr<Conn> c_;
  Reader rd_;
  unsigned long long chunk_left_ = 0;
  long long got_ = 0;
  bool done_ = false;
};
}  // namespace

std::string HttpClientResponse::read_all() {
  std::string out, piece;
  while (next(piece) == kData) out += piece;
  return out;
}

std::unique_ptr<HttpClientResponse> http_open(const std::string& method, const std::string& url, const std::string& body,
                                              const Headers& headers, int timeout_ms, std::string* err,
                                              const TlsClientOptions* tls) {
  Url u;
  if (!Url::parse(url, u)) {
    if (err) *err = "bad url " + url;
    return nullptr;
  }
  auto conn = open_conn(u, timeout_ms, err, tls);
  if (!conn) return nullptr;
  const bool default_port = (u.scheme == "https" && u.port == 443) || (u.scheme == "http" && u.port == 80);
  std::string req = method + " " + u.target() + " HTTP/1.1\r\n";
  if (!headers.count("Host")) req += "Host: " + u.host + (default_port ? "" : ":" + std::to_string(u.port)) + "\r\n";
  bool has_ct = false;
  for (const auto& h : headers) {
    req += h.first + ": " + h.second + "\r\n";
    if (to_lower(h.first) == "content-type") has_ct = true;
  }
  if (!body.empty() && !has_ct) req += "Content-Type: application/json\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n";
  req += body;
  if (!conn->write(req)) {
    if (err) *err = "send failed";
    return nullptr;
  }
  auto resp = std::make_unique<ClientResponse>(std::move(conn));
  std::string line;
  if (!resp->reader().read_line(line)) {
    if (err) *err = "no response (timeout or connection closed)";
    return nullptr;
  }
  auto parts = split(line, ' ', true);
  if (parts.size() < 2 || !starts_with(parts[0], "HTTP/")) {
    if (err) *err = "bad status line";
    return nullptr;
  }
  resp->status = std::atoi(parts[1].c_str());
  if (!read_headers(resp->reader(), resp->headers)) {
    if (err) *err = "truncated response headers";
    return nullptr;
  }
  auto te = resp->headers.find("Transfer-Encoding");
  resp->chunked = te != resp->headers.end() && contains(to_lower(te->second), "chunked");
  auto cl = resp->headers.find("Content-Length");
  if (!resp->chunked && cl != resp->headers.end()) resp->length = std::strtoll(cl->second.c_str(), nullptr, 10);
  if (method == "HEAD" || resp->status == 204 || resp->status == 304) resp->length = 0;
  return resp;
}

std::unique_ptr<RawConn> http_dial(const std::string& url, int timeout_ms, std::string* err, const TlsClientOptions* tls) {
  Url u;
  if (!Url::parse(url, u)) {
    if (err) *err = "bad url " + url;
    return nullptr;
  }
  return open_conn(u, timeout_ms, err, tls);
}

HttpResult http_request(const std::string& method, const std::string& url, const std::string& body,
                        const Headers& headers, int timeout_ms, const TlsClientOptions* tls) {
  HttpResult res;
  auto r = http_open(method, url, body, headers, timeout_ms, &res.error, tls);
  if (!r) return res;
  res.headers = r->headers;
  std::string piece;
  HttpClientResponse::Next n;
  while ((n = r->next(piece)) == HttpClientResponse::kData) res.body += piece;
  if (n != HttpClientResponse::kEnd && res.body.empty() && r->status != 204) res.error = "truncated response";
  res.status = r->status;
  return res;
}

std::pair<long long, long long> pump_bidirectional(RawConn& a, RawConn& b, const std::string& a_pending,
                                                   const std::string& b_pending, int idle_ms) {
  long long ab = 0, ba = 0;
  if (!a_pending.empty()) {
    if (!b.write(a_pending)) return {ab, ba};
    ab += static_cast<long long>(a_pending.size());
  }
  if (!b_pending.empty()) {
    if (!a.write(b_pending)) return {ab, ba};
    ba += static_cast<long long>(b_pending.size());
  }
  // each side's socket waits in poll(); reads never block (bytes are there or TLS has them)
  a.set_timeout_ms(1000);
  b.set_timeout_ms(1000);
  char buf[32768];
  double last = now_seconds();
  for (;;) {
    struct pollfd p[2] = {{a.fd(), POLLIN, 0}, {b.fd(), POLLIN, 0}};
    const bool ra = a.has_buffered(), rb = b.has_buffered();
    int pr = (ra || rb) ? 1 : ::poll(p, 2, 250);
    if (pr < 0 && errno != EINTR) break;
    if (pr == 0) {
      if (idle_ms > 0 && (now_seconds() - last) * 1000 > idle_ms) break;
      continue;
    }
    bool closed = false;
    auto move = [&](RawConn& from, RawConn& to, long long& count) {
      long n = from.read(buf, sizeof buf);
      if (n > 0) {
        if (!to.write(buf, static_cast<size_t>(n))) closed = true;
        count += n;
        last = now_seconds();
      } else if (!(n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))) {
        closed = true;
      }
    };
    if (ra || (p[0].revents & (POLLIN | POLLHUP | POLLERR))) move(a, b, ab);
    if (!closed && (rb || (p[1].revents & (POLLIN | POLLHUP | POLLERR)))) move(b, a, ba);
    if (closed) break;
  }
  return {ab, ba};
}

int http_stream_lines(const std::string& method, const std::string& url, const Headers& headers,
                      const std::function<bool(const std::string&)>& on_line, const std::atomic<bool>* stop,
                      int connect_timeout_ms, std::string* err) {
  auto r = http_open(method, url, "", headers, connect_timeout_ms, err);
  if (!r) return 0;
  r->conn().set_timeout_ms(1000);  // short receive timeout so *stop is observed
  const int status = r->status;
  std::string pending, piece;
  for (;;) {
    if (stop && stop->load()) break;
    const auto n = r->next(piece);
    if (n == HttpClientResponse::kTimeout) continue;
    if (n != HttpClientResponse::kData) break;
    pending += piece;
    size_t nl;
    bool quit = false;
    while ((nl = pending.find('\n')) != std::string::npos) {
      std::string line = pending.substr(0, nl);
      pending.erase(0, nl + 1);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      if (!on_line(line)) {
        quit = true;
        break;
      }
    }
    if (quit) return status;
  }
  if (!trim(pending).empty() && (!stop || !stop->load())) on_line(trim(pending));
  return status;
}

}  // namespace kf
