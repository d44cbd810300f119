// http.h — dependency-free HTTP/1.1 server and client on POSIX sockets.
//
// Server: one accept thread; each connection is served by its own thread (keep-alive, chunked
// responses for long-lived watch streams). Handlers are registered on a Router with
// "/api/{ns}/x" style patterns. Client: blocking requests with timeouts, chunked/Content-Length
// bodies, line streaming for watches, and a pluggable host resolver (used to resolve
// "<svc>.<ns>.svc.<domain>" names through the embedded API server instead of DNS).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kf {

struct CaseLess {
  bool operator()(const std::string& a, const std::string& b) const;
};
using Headers = std::map<std::string, std::string, CaseLess>;

struct HttpRequest {
  std::string method;
  std::string target;  // raw request target
  std::string path;    // decoded path without query
  std::string raw_query;
  Headers headers;
  std::string body;
  std::string remote_addr;
  std::map<std::string, std::vector<std::string>> query;
  std::map<std::string, std::string> params;  // from Router patterns

  std::string header(const std::string& name, const std::string& def = "") const;
  std::string q(const std::string& name, const std::string& def = "") const;
  bool has_q(const std::string& name) const { return query.count(name) > 0; }
  std::string param(const std::string& name) const;
};

class StreamWriter {
 public:
  virtual ~StreamWriter() = default;
  virtual bool write(const std::string& data) = 0;  // one chunk; false once the peer is gone
  virtual bool alive() = 0;
};

struct HttpResponse {
  int status = 200;
  Headers headers;
  std::string body;
  // If set, the server sends headers with chunked encoding and hands the connection to this
  // callback; the response ends when it returns.
  std::function<void(StreamWriter&)> stream;

  void json(int code, const std::string& text) {
    status = code;
    headers["Content-Type"] = "application/json";
    body = text;
  }
  void text(int code, const std::string& t, const std::string& ctype = "text/plain; charset=utf-8") {
    status = code;
    headers["Content-Type"] = ctype;
    body = t;
  }
};

using Handler = std::function<void(HttpRequest&, HttpResponse&)>;

class Router {
 public:
  // pattern: exact "/healthz", parametrised "/kfam/v1/profiles/{profile}", or prefix "/api/*"
  void add(const std::string& method, const std::string& pattern, Handler h);
  void set_not_found(Handler h) { not_found_ = std::move(h); }
  void dispatch(HttpRequest& req, HttpResponse& resp) const;

 private:
  struct Route {
    std::string method;
    std::vector<std::string> segs;
    bool prefix = false;
    Handler h;
  };
  std::vector<Route> routes_;
  Handler not_found_;
};

class HttpServer {
 public:
  HttpServer();
  ~HttpServer();
  void set_handler(Handler h) { handler_ = std::move(h); }
  // port 0 = ephemeral. Returns false (and fills err) if bind/listen fails.
  bool listen(const std::string& addr, int port, std::string* err = nullptr);
  void start();
  void stop();
  int port() const { return port_; }
  std::string address() const { return addr_; }
  size_t active_connections() const { return active_.load(); }

 private:
  void accept_loop(int listen_fd);
  void serve_conn(int fd, std::string remote);
  Handler handler_;
  int listen_fd_ = -1;
  int port_ = 0;
  std::string addr_;
  std::atomic<bool> running_{false};
  std::atomic<size_t> active_{0};
  std::thread accept_thread_;
  std::mutex conns_mu_;
  std::vector<int> conn_fds_;
};

struct HttpResult {
  int status = 0;  // 0 = transport error (see error)
  Headers headers;
  std::string body;
  std::string error;
  bool ok() const { return status >= 200 && status < 300; }
};

struct Url {
  std::string scheme = "http", host, path = "/", query;
  int port = 80;
  static bool parse(const std::string& url, Url& out);
  std::string target() const { return query.empty() ? path : path + "?" + query; }
};

// Resolver hook: map a hostname to "ip:port" (port may be overridden). Return false to fall back
// to the system resolver.
using HostResolver = std::function<bool(const std::string& host, int port, std::string& ip, int& out_port)>;
void set_host_resolver(HostResolver r);

HttpResult http_request(const std::string& method, const std::string& url, const std::string& body = "",
                        const Headers& headers = {}, int timeout_ms = 10000);
// Streams a response body line by line (handles chunked encoding); on_line returning false or
// *stop becoming true ends the stream. Returns the HTTP status (0 on transport error).
int http_stream_lines(const std::string& method, const std::string& url, const Headers& headers,
                      const std::function<bool(const std::string&)>& on_line, const std::atomic<bool>* stop,
                      int connect_timeout_ms = 5000, std::string* err = nullptr);

const char* http_status_text(int code);

}  // namespace kf
