// http.cc — see http.h.
#include "core/http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
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

// ---- socket helpers ---------------------------------------------------------------------------
namespace {

bool send_all(int fd, const char* data, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, data, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    data += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}
bool send_all(int fd, const std::string& s) { return send_all(fd, s.data(), s.size()); }

// Buffered reader over a socket.
class Reader {
 public:
  explicit Reader(int fd) : fd_(fd) {}
  // returns false on EOF/error/timeout
  bool fill() {
    char tmp[16384];
    for (;;) {
      ssize_t r = ::recv(fd_, tmp, sizeof tmp, 0);
      if (r > 0) {
        buf_.append(tmp, static_cast<size_t>(r));
        return true;
      }
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
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
      ssize_t r = ::recv(fd_, tmp, sizeof tmp, 0);
      if (r > 0) {
        out.append(tmp, static_cast<size_t>(r));
        continue;
      }
      if (r < 0 && errno == EINTR) continue;
      return r == 0;
    }
  }

 private:
  void compact() {
    if (pos_ > 65536) {
      buf_.erase(0, pos_);
      pos_ = 0;
    }
  }
  int fd_;
  std::string buf_;
  size_t pos_ = 0;
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
  explicit ChunkWriter(int fd) : fd_(fd) {}
  bool write(const std::string& data) override {
    if (dead_) return false;
    if (data.empty()) return true;
    char hdr[32];
    std::snprintf(hdr, sizeof hdr, "%zx\r\n", data.size());
    if (!send_all(fd_, hdr) || !send_all(fd_, data) || !send_all(fd_, "\r\n")) dead_ = true;
    return !dead_;
  }
  bool alive() override {
    if (dead_) return false;
    struct pollfd p {fd_, POLLIN | POLLRDHUP, 0};
    int r = ::poll(&p, 1, 0);
    if (r > 0 && (p.revents & (POLLHUP | POLLERR | POLLRDHUP))) dead_ = true;
    if (r > 0 && (p.revents & POLLIN)) {
      char c;
      ssize_t n = ::recv(fd_, &c, 1, MSG_PEEK | MSG_DONTWAIT);
      if (n == 0) dead_ = true;
    }
    return !dead_;
  }
  bool finish() { return !dead_ && send_all(fd_, "0\r\n\r\n"); }

 private:
  int fd_;
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

}  // namespace

// ---- server ------------------------------------------------------------------------------------
HttpServer::HttpServer() { ::signal(SIGPIPE, SIG_IGN); }
HttpServer::~HttpServer() { stop(); }

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
  Reader rd(fd);
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
    req.path = url_decode(qm == std::string::npos ? req.target : req.target.substr(0, qm));
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
    std::string head = "HTTP/1.1 " + std::to_string(resp.status) + " " + http_status_text(resp.status) + "\r\n";
    if (resp.stream) {
      for (const auto& h : resp.headers) head += h.first + ": " + h.second + "\r\n";
      head += "Transfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
      if (!send_all(fd, head)) return;
      ChunkWriter w(fd);
      resp.stream(w);
      w.finish();
      return;
    }
    if (!resp.headers.count("Content-Type")) resp.headers["Content-Type"] = "application/json";
    for (const auto& h : resp.headers) head += h.first + ": " + h.second + "\r\n";
    head += "Content-Length: " + std::to_string(resp.body.size()) + "\r\n";
    head += keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
    if (!send_all(fd, head)) return;
    if (req.method != "HEAD" && !send_all(fd, resp.body)) return;
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

HttpResult http_request(const std::string& method, const std::string& url, const std::string& body,
                        const Headers& headers, int timeout_ms) {
  HttpResult res;
  Url u;
  if (!Url::parse(url, u)) {
    res.error = "bad url " + url;
    return res;
  }
  if (u.scheme != "http") {
    res.error = "unsupported scheme " + u.scheme;
    return res;
  }
  int fd = connect_to(u.host, u.port, timeout_ms, &res.error);
  if (fd < 0) return res;
  set_timeouts(fd, timeout_ms);
  std::string req = method + " " + u.target() + " HTTP/1.1\r\nHost: " + u.host + ":" + std::to_string(u.port) + "\r\n";
  bool has_ct = false;
  for (const auto& h : headers) {
    req += h.first + ": " + h.second + "\r\n";
    if (to_lower(h.first) == "content-type") has_ct = true;
  }
  if (!body.empty() && !has_ct) req += "Content-Type: application/json\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n";
  req += body;
  if (!send_all(fd, req)) {
    res.error = "send failed";
    ::close(fd);
    return res;
  }
  Reader rd(fd);
  std::string line;
  if (!rd.read_line(line)) {
    res.error = "no response (timeout or connection closed)";
    ::close(fd);
    return res;
  }
  auto parts = split(line, ' ', true);
  if (parts.size() < 2) {
    res.error = "bad status line";
    ::close(fd);
    return res;
  }
  int status = std::atoi(parts[1].c_str());
  if (!read_headers(rd, res.headers) || !read_body(rd, res.headers, res.body, method != "HEAD")) {
    if (res.body.empty() && status != 204) {
      res.error = "truncated response";
    }
  }
  res.status = status;
  ::close(fd);
  return res;
}

int http_stream_lines(const std::string& method, const std::string& url, const Headers& headers,
                      const std::function<bool(const std::string&)>& on_line, const std::atomic<bool>* stop,
                      int connect_timeout_ms, std::string* err) {
  Url u;
  if (!Url::parse(url, u)) {
    if (err) *err = "bad url";
    return 0;
  }
  int fd = connect_to(u.host, u.port, connect_timeout_ms, err);
  if (fd < 0) return 0;
  set_timeouts(fd, 1000);  // short recv timeout so *stop is observed
  std::string req = method + " " + u.target() + " HTTP/1.1\r\nHost: " + u.host + "\r\n";
  for (const auto& h : headers) req += h.first + ": " + h.second + "\r\n";
  req += "Connection: close\r\n\r\n";
  if (!send_all(fd, req)) {
    ::close(fd);
    return 0;
  }
  std::string buf;
  int status = 0;
  bool headers_done = false, chunked = false;
  std::string pending;  // body bytes not yet split into lines
  size_t chunk_left = 0;
  int cstate = 0;
  char tmp[8192];
  for (;;) {
    if (stop && stop->load()) break;
    ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
    if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) continue;
    if (r <= 0) break;
    buf.append(tmp, static_cast<size_t>(r));
    if (!headers_done) {
      size_t he = buf.find("\r\n\r\n");
      if (he == std::string::npos) continue;
      std::string head = buf.substr(0, he);
      buf.erase(0, he + 4);
      auto lines = split(head, '\n');
      if (!lines.empty()) {
        auto parts = split(trim(lines[0]), ' ', true);
        if (parts.size() >= 2) status = std::atoi(parts[1].c_str());
      }
      for (auto& l : lines)
        if (contains(to_lower(l), "transfer-encoding") && contains(to_lower(l), "chunked")) chunked = true;
      headers_done = true;
    }
    // decode body: chunk state machine (0 = size line, 1 = data, 2 = CRLF after data)
    if (chunked) {
      for (;;) {
        if (cstate == 0) {
          size_t nl = buf.find("\r\n");
          if (nl == std::string::npos) break;
          std::string h = buf.substr(0, nl);
          buf.erase(0, nl + 2);
          if (h.empty()) continue;
          chunk_left = std::strtoul(h.c_str(), nullptr, 16);
          if (chunk_left == 0) goto done;
          cstate = 1;
        } else if (cstate == 1) {
          size_t take = std::min(chunk_left, buf.size());
          if (take == 0) break;
          pending.append(buf, 0, take);
          buf.erase(0, take);
          chunk_left -= take;
          if (chunk_left == 0) cstate = 2;
        } else {
          if (buf.size() < 2) break;
          buf.erase(0, 2);
          cstate = 0;
        }
      }
    } else {
      pending += buf;
      buf.clear();
    }
    size_t nl;
    while ((nl = pending.find('\n')) != std::string::npos) {
      std::string line = pending.substr(0, nl);
      pending.erase(0, nl + 1);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      if (!on_line(line)) goto done;
    }
  }
done:
  if (!pending.empty() && (!stop || !stop->load())) on_line(trim(pending));
  ::close(fd);
  return status;
}

}  // namespace kf
