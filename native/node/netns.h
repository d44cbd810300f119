// netns.h — per-pod network namespaces (kubelet --pod-netns): the isolation the reference gets from
// its CNI + Istio sidecars, on a node whose pods are processes.
//
// A pod's processes run in a network namespace of their own with only a loopback device: nothing
// on the host — no other pod, no host process — can dial a pod's apps, and a pod can dial nothing
// but what the node wires into it:
//   * inbound: the kubelet binds pod_ip:port in the HOST namespace for every TCP containerPort (the
//     pod's enforcement point: NetworkPolicy + Istio AuthorizationPolicy, node/gateway.cc) and
//     connects into the pod namespace to the app behind it;
//   * egress: the node's own endpoints (API server, ingress gateway, mesh listener, KFAM) are
//     relayed: a listener on the same address:port inside the pod namespace, each connection spliced
//     to the host endpoint (EgressRelay). Pod-to-pod traffic therefore always goes through the mesh
//     listener, which authorizes it and records the source pod.
// Kubelet probes, exec and the GPU readiness sidecar's report connect into the namespace directly.
//
// Mechanism: the namespace is created by a helper thread's unshare(CLONE_NEWNET) and kept alive by
// an fd; namespaces are per thread, so a kubelet thread enters one for a connect / posix_spawn
// (NetnsScope) and returns, and processes spawned meanwhile start inside it. This needs
// CAP_SYS_ADMIN (a real kubelet's privilege); without it (an unprivileged node, user namespaces
// disabled) pod_netns_supported() says why and the kubelet falls back to the private-address
// convention (apps on 127.21.x.y behind the inbound listener), which a local process can bypass.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace kf {

// Can this process create and enter network namespaces? Probed once (first call).
bool pod_netns_supported(std::string* why = nullptr);

class PodNetns {
 public:
  // a new network namespace with its loopback device up; nullptr + err on failure
  static std::shared_ptr<PodNetns> create(std::string* err);
  ~PodNetns();
  PodNetns(const PodNetns&) = delete;
  PodNetns& operator=(const PodNetns&) = delete;
  int fd() const { return fd_; }
  // what another process opens to join it (/proc/<kubelet pid>/fd/<fd>): the zygote's children
  std::string path() const;

 private:
  PodNetns() = default;
  int fd_ = -1;
};

// The calling thread is in `ns` for the scope (nullptr: stays where it is), back in the host
// namespace after. Sockets keep the namespace they were created in.
class NetnsScope {
 public:
  explicit NetnsScope(const PodNetns* ns);
  ~NetnsScope();
  NetnsScope(const NetnsScope&) = delete;
  NetnsScope& operator=(const NetnsScope&) = delete;
  bool ok() const { return ok_; }

 private:
  bool entered_ = false, ok_ = true;
};

// The pod a host-side relay connection came from, by the connection's local address (what the
// mesh / ingress listeners see as the peer address).
struct PodSource {
  std::string ns, name;
  std::map<std::string, std::string> labels;
};
bool lookup_pod_source(const std::string& peer_addr, PodSource& out);

// Egress relays of every pod on the node: one epoll thread splices all connections.
class EgressRelay {
 public:
  EgressRelay();
  ~EgressRelay();
  // listeners inside `ns` on each endpoint ("127.0.0.1:6443"), relayed to the same endpoint on the
  // host; returns the endpoints that could not be bound
  std::vector<std::string> add_pod(const std::string& pod_uid, const PodNetns& ns, const std::vector<std::string>& endpoints,
                                   const PodSource& src);
  void remove_pod(const std::string& pod_uid);  // its listeners and open connections
  void stop();
  size_t connections() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace kf
