// odh-notebook-controller — N10: ODH reconciler + the /mutate-notebook-v1 webhook served on
// --webhook-port (default 8443) (reference components/odh-notebook-controller/main.go:74-168).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "odh-notebook-controller";
  s.components = {"odh"};
  s.leader_election_id = "odh-notebook-controller";
  s.default_webhook_port = 8443;
  return kf::run_split(argc, argv, s);
}
