// notebook-controller — N6: Notebook + Culling reconcilers against a remote API server
// (reference components/notebook-controller/main.go:58-148, leader-election ID
// kubeflow-notebook-controller; the culler only runs with ENABLE_CULLING=true).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "notebook-controller";
  s.components = {"notebook", "culler"};
  s.leader_election_id = "kubeflow-notebook-controller";
  return kf::run_split(argc, argv, s);
}
