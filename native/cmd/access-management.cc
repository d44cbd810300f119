// access-management — N19 KFAM REST service on :8081 (reference components/access-management/main.go:36-58;
// flags -userid-header, -userid-prefix, -cluster-admin).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "access-management";
  s.components = {"kfam"};
  s.leader_election_id = "kfam";
  s.default_kfam_port = 8081;
  s.metrics_addr = "0";
  s.probe_addr = "0";
  return kf::run_split(argc, argv, s);
}
