// admission-webhook — N18 PodDefault webhook server (reference components/admission-webhook/main.go,
// HTTPS :4443 there; here HTTP /apply-poddefault plus the MI355X /gpu-readiness and /quota hooks).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "admission-webhook";
  s.components = {"webhooks"};
  s.leader_election_id = "kfamd-admission-webhook";
  s.default_webhook_port = 4443;
  s.metrics_addr = "0";
  return kf::run_split(argc, argv, s);
}
