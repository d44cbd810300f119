// pvcviewer-controller — N17 manager + defaulting/validating webhooks on :9443 (reference
// components/pvcviewer-controller/main.go:55-127).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "pvcviewer-controller";
  s.components = {"pvcviewer"};
  s.leader_election_id = "pvcviewer-controller";
  s.default_webhook_port = 9443;
  return kf::run_split(argc, argv, s);
}
