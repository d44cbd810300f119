// tensorboard-controller — N16 manager (reference components/tensorboard-controller/main.go;
// leader-election ID kubeflow-tensorboard-controller; pod PVC field index set up by the reconciler).
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "tensorboard-controller";
  s.components = {"tensorboard"};
  s.leader_election_id = "kubeflow-tensorboard-controller";
  return kf::run_split(argc, argv, s);
}
