// admission-webhook — N18 PodDefault webhook server (reference components/admission-webhook/main.go:
// HTTPS :4443 from --tlsCertFile / --tlsKeyFile with a certificate watcher), serving
// /apply-poddefault plus the MI355X /gpu-readiness and /quota hooks.
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "admission-webhook";
  s.components = {"webhooks"};
  s.leader_election_id = "kfamd-admission-webhook";
  s.default_webhook_port = 4443;
  s.metrics_addr = "0";
  s.extra_flags = [](kf::Flags& f, kf::ComponentFlags& cf) {
    // the reference's flag names (main.go:755-757); same defaults
    f.add_string("tlsCertFile", &cf.webhook_cert_file, "/etc/webhook/certs/cert.pem", "x509 certificate for HTTPS");
    f.add_string("tlsKeyFile", &cf.webhook_key_file, "/etc/webhook/certs/key.pem", "x509 private key for --tlsCertFile");
    f.add_int("webhookPort", &cf.webhook_port, 4443, "webhook port");
  };
  return kf::run_split(argc, argv, s);
}
