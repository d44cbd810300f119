// http.h — HTTP/1.1 server and client on POSIX sockets, with TLS (OpenSSL 3) on both sides.
//
// Server: one accept thread; each connection is served by its own thread (keep-alive, chunked
// responses for long-lived watch streams, connection hand-over for HTTP Upgrade / WebSocket).
// Handlers are registered on a Router with "/api/{ns}/x" style patterns. HTTPS: enable_tls()
// with a cert/key pair that is re-read when either file changes (the certwatcher behaviour of
// the reference webhooks: admission-webhook/main.go:755-773, config.go:43-60).
// Client: blocking requests with timeouts, chunked/Content-Length bodies, incremental body reads
// (http_open) for streaming proxies, line streaming for watches, https with a CA bundle / PEM
// (hostname-verified, SNI) and optional client certificate, and a pluggable host resolver (used
// to resolve "<svc>.<ns>.svc.<domain>" names through the embedded API server instead of DNS;
// TLS still verifies the original name).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

struct ssl_ctx_st;  // OpenSSL's SSL_CTX

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

// A live byte stream (plain TCP or TLS) — what an Upgrade handler or a tunnel pumps.
class RawConn {
 public:
  virtual ~RawConn() = default;
  // > 0 bytes read; 0 = orderly EOF; < 0 = error or receive timeout (errno EAGAIN)
  virtual long read(char* buf, size_t n) = 0;
  virtual bool write(const char* p, size_t n) = 0;
  bool write(const std::string& s) { return write(s.data(), s.size()); }
  virtual int fd() const = 0;
  // bytes decrypted but not yet read (poll() on fd() does not see them)
  virtual bool has_buffered() const = 0;
  virtual void set_timeout_ms(int ms) = 0;
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
  // If set, the server writes nothing itself: it hands the connection and the bytes already read
  // past this request to the callback (HTTP Upgrade / WebSocket, CONNECT-style tunnels) and closes
  // the connection when it returns.
  std::function<void(RawConn& conn, const std::string& pending)> upgrade;

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

struct TlsServerConfig {
  std::string cert_file, key_file;  // PEM; reloaded when either file's mtime changes
  std::string client_ca_file;       // non-empty: request client certificates verified against it
  bool require_client_cert = false;
};

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
  // Serve HTTPS. Loads the pair now (false + err when it cannot); afterwards a changed file is
  // re-read on the next connection, and a broken replacement keeps the previous pair in service.
  bool enable_tls(const TlsServerConfig& cfg, std::string* err = nullptr);
  bool tls() const { return static_cast<bool>(tls_ctx_); }
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
  std::shared_ptr<::ssl_ctx_st> current_tls_ctx();
  Handler handler_;
  std::mutex tls_mu_;
  std::shared_ptr<::ssl_ctx_st> tls_ctx_;
  TlsServerConfig tls_cfg_;
  long long tls_mtime_ = 0;
  double tls_checked_ = 0;
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

struct TlsClientOptions {
  std::string ca_file;  // PEM bundle; empty (with ca_pem empty) = system trust store
  std::string ca_pem;   // PEM text (a webhook clientConfig.caBundle, decoded)
  std::string cert_file, key_file;  // client certificate (mutual TLS)
  bool insecure_skip_verify = false;
};
// Process-wide defaults for https:// requests that pass no options (in-cluster: the service
// account's ca.crt).
void set_default_tls_client(const TlsClientOptions& o);
TlsClientOptions default_tls_client();

// Resolver hook: map a hostname to "ip:port" (port may be overridden). Return false to fall back
// to the system resolver.
using HostResolver = std::function<bool(const std::string& host, int port, std::string& ip, int& out_port)>;
void set_host_resolver(HostResolver r);

HttpResult http_request(const std::string& method, const std::string& url, const std::string& body = "",
                        const Headers& headers = {}, int timeout_ms = 10000, const TlsClientOptions* tls = nullptr);

// A response whose body is read incrementally (streaming proxies, log follow, watch).
class HttpClientResponse {
 public:
  virtual ~HttpClientResponse() = default;
  int status = 0;
  Headers headers;
  // body framing: Content-Length (length >= 0), chunked, or until EOF
  bool chunked = false;
  long long length = -1;
  enum Next { kData, kEnd, kTimeout, kError };
  // next piece of the de-chunked body
  virtual Next next(std::string& piece) = 0;
  std::string read_all();
  virtual RawConn& conn() = 0;
};
// Sends the request and reads the status line + headers. nullptr on transport error (err set).
std::unique_ptr<HttpClientResponse> http_open(const std::string& method, const std::string& url, const std::string& body,
                                              const Headers& headers, int timeout_ms, std::string* err,
                                              const TlsClientOptions* tls = nullptr);
// Opens a connection (TLS for https://) to the URL's host; for tunnels / Upgrade proxying.
std::unique_ptr<RawConn> http_dial(const std::string& url, int timeout_ms, std::string* err,
                                   const TlsClientOptions* tls = nullptr);
// Bidirectional byte pump between two connections until either side closes (or idle_ms passes
// with no traffic, when > 0). Returns bytes moved a->b and b->a.
std::pair<long long, long long> pump_bidirectional(RawConn& a, RawConn& b, const std::string& a_pending,
                                                   const std::string& b_pending, int idle_ms = 0);
// Streams a response body line by line (handles chunked encoding); on_line returning false or
// *stop becoming true ends the stream. Returns the HTTP status (0 on transport error).
int http_stream_lines(const std::string& method, const std::string& url, const Headers& headers,
                      const std::function<bool(const std::string&)>& on_line, const std::atomic<bool>* stop,
                      int connect_timeout_ms = 5000, std::string* err = nullptr);

const char* http_status_text(int code);

}  // namespace kf
