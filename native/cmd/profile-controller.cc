// profile-controller — N15: Profile reconciler (reference components/profile-controller/main.go:60-127;
// probe port 9876).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "profile-controller";
  s.components = {"profile"};
  s.leader_election_id = "kubeflow-profile-controller";
  s.probe_addr = ":9876";
  return kf::run_split(argc, argv, s);
}
