// http_test.cc — HTTP/1.1 server + client, streaming, Upgrade hand-over, TLS with an in-process
// generated certificate (OpenSSL API: EC P-256 key, self-signed, SAN IP:127.0.0.1).
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/x509v3.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>

#include "core/http.h"
#include "core/util.h"
#include "tests/harness.h"

long long now_unix_ms_for_serial();

namespace {

std::string tmpdir() {
  char tmpl[] = "/tmp/kfamd-http-test-XXXXXX";
  return ::mkdtemp(tmpl) ? std::string(tmpl) : std::string("/tmp");
}

// self-signed certificate + key for subjectAltName `san` ("IP:127.0.0.1"); PEM files under dir
bool make_cert(const std::string& dir, const std::string& san, std::string& cert_pem) {
  EVP_PKEY* key = EVP_EC_gen("P-256");
  if (!key) return false;
  X509* x = X509_new();
  ASN1_INTEGER_set(X509_get_serialNumber(x), static_cast<long>(now_unix_ms_for_serial()));
  X509_gmtime_adj(X509_getm_notBefore(x), -60);
  X509_gmtime_adj(X509_getm_notAfter(x), 3600);
  X509_set_pubkey(x, key);
  X509_NAME* n = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(n, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("kfamd-test"), -1, -1, 0);
  X509_set_issuer_name(x, n);
  X509V3_CTX ctx;
  X509V3_set_ctx_nodb(&ctx);
  X509V3_set_ctx(&ctx, x, x, nullptr, nullptr, 0);
  for (auto [nid, val] : {std::pair<int, std::string>{NID_subject_alt_name, san}, {NID_basic_constraints, "critical,CA:TRUE"}}) {
    X509_EXTENSION* e = X509V3_EXT_conf_nid(nullptr, &ctx, nid, val.c_str());
    X509_add_ext(x, e, -1);
    X509_EXTENSION_free(e);
  }
  X509_sign(x, key, EVP_sha256());
  FILE* f = std::fopen((dir + "/tls.crt").c_str(), "w");
  PEM_write_X509(f, x);
  std::fclose(f);
  f = std::fopen((dir + "/tls.key").c_str(), "w");
  PEM_write_PrivateKey(f, key, nullptr, nullptr, 0, nullptr, nullptr);
  std::fclose(f);
  X509_free(x);
  EVP_PKEY_free(key);
  return kf::read_file(dir + "/tls.crt", cert_pem);
}

}  // namespace

long long now_unix_ms_for_serial() { return kf::now_unix_ms() & 0x7fffffff; }

TEST(http, request_response_keepalive_and_stream) {
  kf::HttpServer srv;
  REQUIRE(srv.listen("127.0.0.1", 0));
  srv.set_handler([](kf::HttpRequest& req, kf::HttpResponse& resp) {
    if (req.path == "/stream") {
      resp.headers["Content-Type"] = "text/plain";
      resp.stream = [](kf::StreamWriter& w) {
        for (int i = 0; i < 3; ++i) w.write("line" + std::to_string(i) + "\n");
      };
      return;
    }
    resp.json(200, "{\"path\":\"" + req.path + "\",\"q\":\"" + req.q("x") + "\",\"len\":" + std::to_string(req.body.size()) + "}");
  });
  srv.start();
  const std::string base = "http://127.0.0.1:" + std::to_string(srv.port());
  kf::HttpResult r = kf::http_request("POST", base + "/echo?x=1", std::string(100000, 'a'));
  REQUIRE(r.ok());
  CHECK_EQ(r.body, std::string("{\"path\":\"/echo\",\"q\":\"1\",\"len\":100000}"));
  std::vector<std::string> lines;
  CHECK_EQ(kf::http_stream_lines("GET", base + "/stream", {}, [&](const std::string& l) { lines.push_back(l); return true; },
                                 nullptr), 200);
  CHECK(lines == std::vector<std::string>({"line0", "line1", "line2"}));
  std::string err;
  auto o = kf::http_open("GET", base + "/stream", "", {}, 5000, &err);
  REQUIRE(o);
  CHECK(o->chunked);
  CHECK_EQ(o->read_all(), std::string("line0\nline1\nline2\n"));
  srv.stop();
}

TEST(http, upgrade_hands_over_the_connection) {
  kf::HttpServer srv;
  REQUIRE(srv.listen("127.0.0.1", 0));
  srv.set_handler([](kf::HttpRequest&, kf::HttpResponse& resp) {
    resp.upgrade = [](kf::RawConn& c, const std::string& pending) {
      c.write(std::string("HTTP/1.1 101 Switching Protocols\r\nUpgrade: echo\r\nConnection: Upgrade\r\n\r\n"));
      std::string got = pending;
      char buf[256];
      while (got.size() < 5) {
        long n = c.read(buf, sizeof buf);
        if (n <= 0) return;
        got.append(buf, static_cast<size_t>(n));
      }
      c.write("echo:" + got);
    };
  });
  srv.start();
  std::string err;
  auto c = kf::http_dial("http://127.0.0.1:" + std::to_string(srv.port()) + "/", 5000, &err);
  REQUIRE(c);
  c->write(std::string("GET / HTTP/1.1\r\nHost: x\r\nConnection: Upgrade\r\nUpgrade: echo\r\n\r\nhel"));
  c->write(std::string("lo"));
  std::string got;
  char buf[512];
  while (got.find("echo:hello") == std::string::npos) {
    long n = c->read(buf, sizeof buf);
    if (n <= 0) break;
    got.append(buf, static_cast<size_t>(n));
  }
  CHECK(got.find(" 101 ") != std::string::npos);
  CHECK(got.find("echo:hello") != std::string::npos);
  srv.stop();
}

TEST(http, tls_server_and_verifying_client) {
  const std::string dir = tmpdir();
  std::string pem;
  REQUIRE(make_cert(dir, "IP:127.0.0.1", pem));
  kf::HttpServer srv;
  std::string err;
  REQUIRE(srv.enable_tls(kf::TlsServerConfig{dir + "/tls.crt", dir + "/tls.key", "", false}, &err));
  REQUIRE(srv.listen("127.0.0.1", 0));
  srv.set_handler([](kf::HttpRequest& req, kf::HttpResponse& resp) { resp.text(200, "secure " + req.path); });
  srv.start();
  const std::string url = "https://127.0.0.1:" + std::to_string(srv.port()) + "/x";
  kf::TlsClientOptions trust;
  trust.ca_pem = pem;
  kf::HttpResult ok = kf::http_request("GET", url, "", {}, 5000, &trust);
  CHECK_EQ(ok.status, 200);
  CHECK_EQ(ok.body, std::string("secure /x"));
  kf::TlsClientOptions system;  // system trust store: our test CA is not in it
  kf::HttpResult refused = kf::http_request("GET", url, "", {}, 5000, &system);
  CHECK_EQ(refused.status, 0);
  CHECK(refused.error.find("certificate verify failed") != std::string::npos);
  // the certificate names 127.0.0.1 only: "localhost" fails hostname verification
  kf::HttpResult wrong_host =
      kf::http_request("GET", "https://localhost:" + std::to_string(srv.port()) + "/x", "", {}, 5000, &trust);
  CHECK_EQ(wrong_host.status, 0);
  kf::TlsClientOptions insecure;
  insecure.insecure_skip_verify = true;
  CHECK_EQ(kf::http_request("GET", url, "", {}, 5000, &insecure).status, 200);
  // plain HTTP against the TLS port gets no HTTP response
  CHECK_EQ(kf::http_request("GET", "http://127.0.0.1:" + std::to_string(srv.port()) + "/x", "", {}, 2000).status, 0);
  srv.stop();
}
