// kfamd-node — one MI355X node joined to a remote kube-lite API server: GPU-topology-aware
// scheduler, built-in workload controllers, the process-pod kubelet (device plugin + xGMI placement)
// and the ingress gateway. Several kfamd-node processes (distinct --node-name / --pod-cidr-prefix)
// simulate a multi-node cluster on one host.
#include "cmd/split_main.h"

int main(int argc, char** argv) {
  kf::SplitSpec s;
  s.name = "kfamd-node";
  s.components = {"builtin", "scheduler", "kubelet", "gateway"};
  s.leader_election_id = "kfamd-node";
  s.metrics_addr = "0";
  s.probe_addr = "0";
  return kf::run_split(argc, argv, s);
}
