// netns.cc — see netns.h.
#include "node/netns.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <net/if.h>
#include <netinet/in.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>

#include "core/util.h"

namespace kf {

namespace {
// the host namespace, opened by the first caller (the kubelet's constructor, on the main thread)
int host_netns_fd() {
  static const int fd = ::open("/proc/self/ns/net", O_RDONLY | O_CLOEXEC);
  return fd;
}

bool loopback_up(std::string* err) {
  const int s = ::socket(AF_INET, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (s < 0) {
    if (err) *err = std::string("socket: ") + std::strerror(errno);
    return false;
  }
  ifreq ifr{};
  std::strncpy(ifr.ifr_name, "lo", IFNAMSIZ - 1);
  bool ok = ::ioctl(s, SIOCGIFFLAGS, &ifr) == 0;
  if (ok) {
    ifr.ifr_flags = static_cast<short>(ifr.ifr_flags | IFF_UP | IFF_RUNNING);
    ok = ::ioctl(s, SIOCSIFFLAGS, &ifr) == 0;
  }
  if (!ok && err) *err = std::string("bring up lo: ") + std::strerror(errno);
  ::close(s);
  return ok;
}

bool split_endpoint(const std::string& ep, sockaddr_in& sa) {
  const size_t colon = ep.rfind(':');
  if (colon == std::string::npos) return false;
  std::memset(&sa, 0, sizeof sa);
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(std::atoi(ep.c_str() + colon + 1)));
  return ::inet_pton(AF_INET, ep.substr(0, colon).c_str(), &sa.sin_addr) == 1 && sa.sin_port != 0;
}

std::string local_addr(int fd) {
  sockaddr_in sa{};
  socklen_t len = sizeof sa;
  if (::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len) != 0) return "";
  char ip[INET_ADDRSTRLEN] = {0};
  ::inet_ntop(AF_INET, &sa.sin_addr, ip, sizeof ip);
  return std::string(ip) + ":" + std::to_string(ntohs(sa.sin_port));
}

std::mutex& sources_mu() {
  static std::mutex m;
  return m;
}
std::map<std::string, PodSource>& sources() {
  static std::map<std::string, PodSource> m;
  return m;
}
}  // namespace

bool pod_netns_supported(std::string* why) {
  static const std::pair<bool, std::string> probe = [] {
    if (host_netns_fd() < 0) return std::make_pair(false, std::string("cannot open /proc/self/ns/net"));
    std::string err;
    auto ns = PodNetns::create(&err);
    if (!ns) return std::make_pair(false, err);
    NetnsScope in(ns.get());
    if (!in.ok()) return std::make_pair(false, std::string("setns into a pod namespace: ") + std::strerror(errno));
    return std::make_pair(true, std::string());
  }();
  if (why) *why = probe.second;
  return probe.first;
}

std::shared_ptr<PodNetns> PodNetns::create(std::string* err) {
  int fd = -1;
  std::string e;
  // a throwaway thread: unshare() moves only the calling thread, which then ends; the fd keeps the
  // namespace alive
  std::thread t([&] {
    if (::unshare(CLONE_NEWNET) != 0) {
      e = std::string("unshare(CLONE_NEWNET): ") + std::strerror(errno);
      return;
    }
    if (!loopback_up(&e)) return;
    fd = ::open("/proc/thread-self/ns/net", O_RDONLY | O_CLOEXEC);
    if (fd < 0) e = std::string("open /proc/thread-self/ns/net: ") + std::strerror(errno);
  });
  t.join();
  if (fd < 0) {
    if (err) *err = e;
    return nullptr;
  }
  std::shared_ptr<PodNetns> ns(new PodNetns());
  ns->fd_ = fd;
  return ns;
}

PodNetns::~PodNetns() {
  if (fd_ >= 0) ::close(fd_);
}

std::string PodNetns::path() const { return "/proc/" + std::to_string(::getpid()) + "/fd/" + std::to_string(fd_); }

NetnsScope::NetnsScope(const PodNetns* ns) {
  if (!ns) return;
  ok_ = ::setns(ns->fd(), CLONE_NEWNET) == 0;
  entered_ = ok_;
}

NetnsScope::~NetnsScope() {
  if (entered_ && ::setns(host_netns_fd(), CLONE_NEWNET) != 0) std::abort();  // a thread stranded in a pod
}

bool lookup_pod_source(const std::string& peer_addr, PodSource& out) {
  std::lock_guard<std::mutex> g(sources_mu());
  auto it = sources().find(peer_addr);
  if (it == sources().end()) return false;
  out = it->second;
  return true;
}

// ---- egress relay ---------------------------------------------------------------------------------
struct EgressRelay::Impl {
  struct Listener {
    std::string pod;
    sockaddr_in target{};
    PodSource src;
  };
  struct Conn {
    int peer = -1;
    std::string pod, source_key;  // source_key: the host-side socket's address (lookup_pod_source)
    std::string out;              // bytes read from the peer, not yet written here
    bool eof_in = false;          // this side sent EOF
    bool shut = false;            // we shut down this side's write half
  };
  int ep = -1, wake = -1;
  std::atomic<bool> running{true};
  mutable std::mutex mu;
  std::map<int, Listener> listeners;
  std::map<int, Conn> conns;
  std::thread th;

  void arm(int fd) {  // caller holds mu
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    const Conn& c = it->second;
    auto p = conns.find(c.peer);
    uint32_t ev = 0;
    if (!c.eof_in && p != conns.end() && p->second.out.empty()) ev |= EPOLLIN;  // backpressure
    if (!c.out.empty()) ev |= EPOLLOUT;
    epoll_event e{};
    e.events = ev;
    e.data.fd = fd;
    ::epoll_ctl(ep, EPOLL_CTL_MOD, fd, &e);
  }
  void close_conn(int fd) {  // both halves of the pair
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    const int peer = it->second.peer;
    for (int f : {fd, peer}) {
      auto c = conns.find(f);
      if (c == conns.end()) continue;
      if (!c->second.source_key.empty()) {
        std::lock_guard<std::mutex> g(sources_mu());
        sources().erase(c->second.source_key);
      }
      ::close(f);
      conns.erase(c);
    }
  }
  void accept_one(int lfd) {
    const Listener& l = listeners[lfd];
    const int in = ::accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (in < 0) return;
    const int out = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);  // this thread: host namespace
    if (out < 0 || ::connect(out, reinterpret_cast<const sockaddr*>(&l.target), sizeof l.target) != 0) {
      if (out >= 0) ::close(out);
      ::close(in);
      return;
    }
    ::fcntl(out, F_SETFL, ::fcntl(out, F_GETFL) | O_NONBLOCK);
    Conn a, b;
    a.peer = out;
    b.peer = in;
    a.pod = b.pod = l.pod;
    b.source_key = local_addr(out);
    {
      std::lock_guard<std::mutex> g(sources_mu());
      sources()[b.source_key] = l.src;
    }
    conns[in] = a;
    conns[out] = b;
    for (int f : {in, out}) {
      epoll_event e{};
      e.events = EPOLLIN;
      e.data.fd = f;
      ::epoll_ctl(ep, EPOLL_CTL_ADD, f, &e);
    }
  }
  void on_readable(int fd) {
    Conn& c = conns[fd];
    Conn& p = conns[c.peer];
    char buf[65536];
    const ssize_t n = ::read(fd, buf, sizeof buf);
    if (n < 0 && (errno == EAGAIN || errno == EINTR)) return;
    if (n <= 0) {
      c.eof_in = true;
      if (n < 0 || (p.eof_in && p.out.empty() && c.out.empty())) {
        close_conn(fd);
        return;
      }
      if (p.out.empty() && !p.shut) {
        ::shutdown(c.peer, SHUT_WR);
        p.shut = true;
      }
      arm(fd);
      return;
    }
    ssize_t w = ::send(c.peer, buf, static_cast<size_t>(n), MSG_NOSIGNAL);
    if (w < 0 && errno != EAGAIN) {
      close_conn(fd);
      return;
    }
    if (w < 0) w = 0;
    if (w < n) p.out.append(buf + w, static_cast<size_t>(n - w));
    arm(fd);
    arm(c.peer);
  }
  void on_writable(int fd) {
    Conn& c = conns[fd];
    const ssize_t w = ::send(fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
    if (w < 0 && errno != EAGAIN) {
      close_conn(fd);
      return;
    }
    if (w > 0) c.out.erase(0, static_cast<size_t>(w));
    Conn& p = conns[c.peer];
    if (c.out.empty() && p.eof_in && !c.shut) {
      ::shutdown(fd, SHUT_WR);
      c.shut = true;
      if (c.eof_in && p.out.empty()) {  // both directions ended and flushed
        close_conn(fd);
        return;
      }
    }
    arm(fd);
    arm(c.peer);
  }
  void loop() {
    epoll_event evs[64];
    while (running) {
      const int n = ::epoll_wait(ep, evs, 64, 500);
      std::lock_guard<std::mutex> g(mu);
      for (int i = 0; i < n; ++i) {
        const int fd = evs[i].data.fd;
        if (fd == wake) continue;
        if (listeners.count(fd)) {
          accept_one(fd);
          continue;
        }
        if (!conns.count(fd)) continue;  // closed earlier in this batch
        if (evs[i].events & (EPOLLERR | EPOLLHUP) && !(evs[i].events & (EPOLLIN | EPOLLOUT))) {
          close_conn(fd);
          continue;
        }
        if (evs[i].events & EPOLLIN) on_readable(fd);
        if (conns.count(fd) && (evs[i].events & EPOLLOUT)) on_writable(fd);
      }
    }
  }
};

EgressRelay::EgressRelay() : impl_(std::make_unique<Impl>()) {
  impl_->ep = ::epoll_create1(EPOLL_CLOEXEC);
  impl_->wake = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  epoll_event e{};
  e.events = EPOLLIN;
  e.data.fd = impl_->wake;
  ::epoll_ctl(impl_->ep, EPOLL_CTL_ADD, impl_->wake, &e);
  impl_->th = std::thread([this] { impl_->loop(); });
}

EgressRelay::~EgressRelay() {
  stop();
  if (impl_->ep >= 0) ::close(impl_->ep);
  if (impl_->wake >= 0) ::close(impl_->wake);
}

void EgressRelay::stop() {
  if (!impl_->running.exchange(false)) return;
  const uint64_t one = 1;
  (void)!::write(impl_->wake, &one, sizeof one);
  if (impl_->th.joinable()) impl_->th.join();
  std::lock_guard<std::mutex> g(impl_->mu);
  for (auto& kv : impl_->listeners) ::close(kv.first);
  impl_->listeners.clear();
  while (!impl_->conns.empty()) impl_->close_conn(impl_->conns.begin()->first);
}

std::vector<std::string> EgressRelay::add_pod(const std::string& pod_uid, const PodNetns& ns,
                                              const std::vector<std::string>& endpoints, const PodSource& src) {
  std::vector<std::string> failed;
  for (const auto& ep : endpoints) {
    Impl::Listener l;
    if (!split_endpoint(ep, l.target)) {
      failed.push_back(ep);
      continue;
    }
    l.pod = pod_uid;
    l.src = src;
    int fd;
    {
      NetnsScope in(&ns);
      fd = in.ok() ? ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0) : -1;
    }
    const int one = 1;
    if (fd < 0 || ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one) != 0 ||
        ::bind(fd, reinterpret_cast<const sockaddr*>(&l.target), sizeof l.target) != 0 || ::listen(fd, 128) != 0) {
      if (fd >= 0) ::close(fd);
      failed.push_back(ep);
      continue;
    }
    std::lock_guard<std::mutex> g(impl_->mu);
    impl_->listeners[fd] = l;
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.fd = fd;
    ::epoll_ctl(impl_->ep, EPOLL_CTL_ADD, fd, &e);
  }
  return failed;
}

void EgressRelay::remove_pod(const std::string& pod_uid) {
  std::lock_guard<std::mutex> g(impl_->mu);
  for (auto it = impl_->listeners.begin(); it != impl_->listeners.end();) {
    if (it->second.pod != pod_uid) {
      ++it;
      continue;
    }
    ::close(it->first);
    it = impl_->listeners.erase(it);
  }
  std::vector<int> fds;
  for (const auto& kv : impl_->conns)
    if (kv.second.pod == pod_uid) fds.push_back(kv.first);
  for (int fd : fds) impl_->close_conn(fd);
}

size_t EgressRelay::connections() const {
  std::lock_guard<std::mutex> g(impl_->mu);
  return impl_->conns.size() / 2;
}

}  // namespace kf
