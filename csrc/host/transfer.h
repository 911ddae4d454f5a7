// transfer.h — TCP message transport + RPC layer for the host control plane
// and CPU clusters.
//
// Reference: core/transfer/{Listener,Route,transfer}.h + core/Message.h +
// core/common.h (ZeroMQ PUSH/PULL full mesh, 2-frame messages, message-class
// handler registry, msg-id callbacks, deferred replies).  ZeroMQ is not a
// dependency here: plain POSIX TCP with length-prefixed frames.
//
// Semantics kept from the reference:
//   * MetaMessage {message_class, addr, client_id, message_id}; a response is
//     marked by message_class == -1 (Message.h:175-176);
//   * `send(req, to_id)` assigns message_id = counter++ and stores the
//     callback, which runs when the response arrives (transfer.h:75-112,183-208);
//   * handlers run on an async pool; the response is sent ONLY if its payload
//     is non-empty — an empty response defers the reply (transfer.h:154-179),
//     which the master uses for registration;
//   * nodes are addressed by integer ids registered with their address
//     (Route.h:31-79); master = 0, servers 1..S, workers INT_MAX-1, -2, ...
// Fixes: the handler registry is locked (transfer.h:41-45 is not), the
// receive path copies message bytes (Message.h:156 reads the zmq_msg_t
// struct itself), shutdown closes sockets instead of self-poking.
#pragma once
#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "buffer.h"
#include "channel.h"
#include "common.h"
#include "string_util.h"

namespace ss {

// ------------------------------------------------------------------ address
struct Addr {
  std::string ip = "127.0.0.1";
  uint16_t port = 0;
  Addr() = default;
  Addr(std::string i, uint16_t p) : ip(std::move(i)), port(p) {}
  // "tcp://1.2.3.4:5678" or "1.2.3.4:5678"
  static Addr parse(const std::string& s) {
    std::string t = s;
    if (startswith(t, "tcp://")) t = t.substr(6);
    const size_t c = t.rfind(':');
    SS_CHECK_MSG(c != std::string::npos, "bad address: " << s);
    return Addr(t.substr(0, c), (uint16_t)std::stoi(t.substr(c + 1)));
  }
  std::string to_string() const { return "tcp://" + ip + ":" + std::to_string(port); }
  uint32_t ip4() const {
    in_addr a{};
    SS_CHECK_MSG(inet_pton(AF_INET, ip.c_str(), &a) == 1, "bad ipv4: " << ip);
    return a.s_addr;
  }
  static Addr from_ip4(uint32_t ip4, uint16_t port) {
    char buf[INET_ADDRSTRLEN];
    in_addr a{};
    a.s_addr = ip4;
    inet_ntop(AF_INET, &a, buf, sizeof(buf));
    return Addr(buf, port);
  }
  bool operator==(const Addr& o) const { return ip == o.ip && port == o.port; }
};

// last non-loopback IPv4 (reference get_local_ip, core/common.h:87-113);
// SS_LOCAL_IP overrides, 127.0.0.1 if none.
inline std::string get_local_ip() {
  if (const char* e = std::getenv("SS_LOCAL_IP")) return e;
  std::string ip = "127.0.0.1";
  ifaddrs* ifs = nullptr;
  if (getifaddrs(&ifs) == 0) {
    for (ifaddrs* p = ifs; p; p = p->ifa_next) {
      if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
      char buf[INET_ADDRSTRLEN];
      inet_ntop(AF_INET, &((sockaddr_in*)p->ifa_addr)->sin_addr, buf, sizeof(buf));
      if (std::string(buf) != "127.0.0.1") ip = buf;
    }
    freeifaddrs(ifs);
  }
  return ip;
}

// ------------------------------------------------------------------ message
#pragma pack(push, 1)
struct MetaMessage {
  int32_t message_class = 0;
  int32_t client_id = -3;    // -3 unset, -1 worker, -2 server (Message.h:18-38)
  int64_t message_id = -1;
  uint32_t ip4 = 0;          // sender's listen address
  uint16_t port = 0;
  uint16_t pad = 0;
};
#pragma pack(pop)
static_assert(sizeof(MetaMessage) == 24, "MetaMessage must stay 24 bytes");

enum : int32_t { kResponseClass = -1 };

struct Request {
  MetaMessage meta;
  BinaryBuffer cont;
  std::function<void(std::shared_ptr<Request>)> call_back_handler;
  bool is_response() const { return meta.message_class == kResponseClass; }
  void set_worker() { meta.client_id = -1; }
  void set_server() { meta.client_id = -2; }
};

// Reference message classes (core/system/message_classes.h:13-42).
enum MsgClass : int32_t {
  NODE_INIT_ADDRESS = 0,
  NODE_ASKFOR_HASHFRAG = 1,
  WORKER_PULL_REQUEST = 2,
  WORKER_PUSH_REQUEST = 3,
  WORKER_FINISH_WORK = 4,
  SERVER_TOLD_TO_TERMINATE = 5,
  USER_MESSAGE_BASE = 64,
};

// ------------------------------------------------------------------ sockets
namespace net {
inline void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
inline bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;  // reference ignore_signal_call, common.h:27-38
      return false;
    }
    c += w;
    n -= (size_t)w;
  }
  return true;
}
inline bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    const ssize_t r = ::recv(fd, c, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}
inline int connect_to(const Addr& a, double timeout_s = 30.0) {
  Timer t;
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    SS_CHECK(fd >= 0);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(a.port);
    sa.sin_addr.s_addr = a.ip4();
    if (::connect(fd, (sockaddr*)&sa, sizeof(sa)) == 0) {
      set_nodelay(fd);
      return fd;
    }
    ::close(fd);
    SS_CHECK_MSG(t.elapsed() < timeout_s, "connect to " << a.to_string() << " timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}
}  // namespace net

// ------------------------------------------------------------------ transfer
class Transfer : NonCopyable {
 public:
  using Handler = std::function<void(std::shared_ptr<Request> req, Request& rsp)>;

  Transfer() = default;
  ~Transfer() { service_end(); }

  // bind to addr ("" / port 0 => random port on the local IP)
  void listen(const std::string& addr = "") {
    SS_CHECK_MSG(lfd_ < 0, "already listening");
    Addr a = addr.empty() ? Addr(get_local_ip(), 0) : Addr::parse(addr);
    lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    SS_CHECK(lfd_ >= 0);
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(a.port);
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    SS_CHECK_MSG(::bind(lfd_, (sockaddr*)&sa, sizeof(sa)) == 0,
                 "bind " << a.to_string() << ": " << std::strerror(errno));
    SS_CHECK(::listen(lfd_, 128) == 0);
    socklen_t len = sizeof(sa);
    getsockname(lfd_, (sockaddr*)&sa, &len);
    addr_ = Addr(a.ip, ntohs(sa.sin_port));
  }

  // start the accept loop and `async_threads` handler threads
  void service_start(int async_threads = 4) {
    SS_CHECK_MSG(lfd_ >= 0, "listen() first");
    SS_CHECK(!running_.exchange(true));
    pool_.reset(new ThreadPool(async_threads));
    const int lfd = lfd_;  // the accept thread never reads the member (service_end resets it)
    accept_thread_ = std::thread([this, lfd] { accept_loop(lfd); });
  }

  void service_end() {
    if (!running_.exchange(false)) {
      if (lfd_ >= 0) {
        ::close(lfd_);
        lfd_ = -1;
      }
      return;
    }
    ::shutdown(lfd_, SHUT_RDWR);  // wakes accept(); close only after the join so the
    if (accept_thread_.joinable()) accept_thread_.join();  // fd number cannot be reused under it
    ::close(lfd_);
    lfd_ = -1;
    {
      std::lock_guard<std::mutex> lk(conn_mu_);
      for (auto& kv : out_) {
        ::shutdown(kv.second->fd, SHUT_RDWR);
        ::close(kv.second->fd);
      }
      out_.clear();
      for (int fd : in_fds_) ::shutdown(fd, SHUT_RDWR);
    }
    for (auto& t : readers_)
      if (t.joinable()) t.join();
    readers_.clear();
    {
      std::lock_guard<std::mutex> lk(conn_mu_);
      for (int fd : in_fds_) ::close(fd);
      in_fds_.clear();
    }
    if (pool_) pool_->stop();
  }

  const Addr& addr() const { return addr_; }
  int client_id() const { return client_id_; }
  void set_client_id(int id) { client_id_ = id; }

  // ---- route (reference BaseRoute)
  void register_node(int id, const Addr& a) {
    std::unique_lock<std::shared_mutex> lk(route_mu_);
    route_[id] = a;
  }
  bool delete_node(int id) {
    std::unique_lock<std::shared_mutex> lk(route_mu_);
    {
      std::lock_guard<std::mutex> lk2(conn_mu_);
      auto it = out_.find(id);
      if (it != out_.end()) {
        ::close(it->second->fd);
        out_.erase(it);
      }
    }
    return route_.erase(id) != 0;
  }
  bool has_node(int id) const {
    std::shared_lock<std::shared_mutex> lk(route_mu_);
    return route_.count(id) != 0;
  }
  Addr node_addr(int id) const {
    std::shared_lock<std::shared_mutex> lk(route_mu_);
    auto it = route_.find(id);
    SS_CHECK_MSG(it != route_.end(), "unknown node id " << id);
    return it->second;
  }
  std::map<int, Addr> route() const {
    std::shared_lock<std::shared_mutex> lk(route_mu_);
    return route_;
  }

  // ---- message classes
  void add_handler(int32_t msg_class, Handler h) {
    std::unique_lock<std::shared_mutex> lk(handler_mu_);
    handlers_[msg_class] = std::move(h);
  }
  bool has_handler(int32_t c) const {
    std::shared_lock<std::shared_mutex> lk(handler_mu_);
    return handlers_.count(c) != 0;
  }

  // ---- send
  int64_t send(Request&& req, int to_id) {
    const int64_t id = msg_counter_.fetch_add(1);
    req.meta.message_id = id;
    if (req.meta.client_id == -3) req.meta.client_id = client_id_;
    stamp(req.meta);
    if (req.call_back_handler) {
      std::lock_guard<std::mutex> lk(cb_mu_);
      callbacks_[id] = std::move(req.call_back_handler);
    }
    deliver(to_id, node_addr(to_id), req);
    return id;
  }
  void send_response(Request&& rsp, int to_id) {
    rsp.meta.message_class = kResponseClass;
    stamp(rsp.meta);
    deliver(to_id, node_addr(to_id), rsp);
  }
  void send_response_to(Request&& rsp, const Addr& a) {
    rsp.meta.message_class = kResponseClass;
    stamp(rsp.meta);
    deliver(INT32_MIN, a, rsp);
  }
  size_t pending_callbacks() const {
    std::lock_guard<std::mutex> lk(cb_mu_);
    return callbacks_.size();
  }

 private:
  struct Conn {
    int fd;
    std::mutex mu;
  };

  void stamp(MetaMessage& m) const {
    m.ip4 = addr_.ip4();
    m.port = addr_.port;
  }

  std::shared_ptr<Conn> conn_for(int id, const Addr& a) {
    std::lock_guard<std::mutex> lk(conn_mu_);
    const int key = id == INT32_MIN ? (int)(0x40000000 ^ a.port ^ (a.ip4() << 8)) : id;
    auto it = out_.find(key);
    if (it != out_.end()) return it->second;
    auto c = std::make_shared<Conn>();
    c->fd = net::connect_to(a);
    out_[key] = c;
    return c;
  }

  void deliver(int id, const Addr& a, const Request& r) {
    auto c = conn_for(id, a);
    const uint32_t len = (uint32_t)(sizeof(MetaMessage) + r.cont.size());
    std::lock_guard<std::mutex> lk(c->mu);  // per-destination send lock (Route.h:66-79)
    SS_CHECK_MSG(net::write_all(c->fd, &len, 4) && net::write_all(c->fd, &r.meta, sizeof(r.meta)) &&
                     net::write_all(c->fd, r.cont.data(), r.cont.size()),
                 "send to node " << id << " failed");
  }

  void accept_loop(int lfd) {
    while (running_) {
      sockaddr_in sa{};
      socklen_t len = sizeof(sa);
      const int fd = ::accept(lfd, (sockaddr*)&sa, &len);
      if (fd < 0) {
        if (!running_) break;
        if (errno == EINTR) continue;
        break;
      }
      net::set_nodelay(fd);
      std::lock_guard<std::mutex> lk(conn_mu_);
      in_fds_.push_back(fd);
      readers_.emplace_back([this, fd] { read_loop(fd); });
    }
  }

  void read_loop(int fd) {
    for (;;) {
      uint32_t len = 0;
      if (!net::read_all(fd, &len, 4)) return;
      if (len < sizeof(MetaMessage)) return;
      auto req = std::make_shared<Request>();
      if (!net::read_all(fd, &req->meta, sizeof(MetaMessage))) return;
      const size_t body = len - sizeof(MetaMessage);
      req->cont.bytes().resize(body);
      if (body && !net::read_all(fd, req->cont.data(), body)) return;
      if (req->is_response())
        handle_response(std::move(req));
      else
        handle_request(std::move(req));
    }
  }

  void handle_request(std::shared_ptr<Request> req) {
    Handler h;
    {
      std::shared_lock<std::shared_mutex> lk(handler_mu_);
      auto it = handlers_.find(req->meta.message_class);
      if (it != handlers_.end()) h = it->second;
    }
    if (!h) {
      SS_LOG_ERROR("no handler for message class %d", req->meta.message_class);
      return;
    }
    pool_->submit([this, req, h] {
      Request rsp;
      rsp.meta.message_id = req->meta.message_id;
      rsp.meta.client_id = client_id_;
      h(req, rsp);
      // deferred reply: an empty response is not sent (transfer.h:173-177)
      if (rsp.cont.size() > 0) {
        rsp.meta.message_id = req->meta.message_id;
        send_response_to(std::move(rsp), Addr::from_ip4(req->meta.ip4, req->meta.port));
      }
    });
  }

  void handle_response(std::shared_ptr<Request> rsp) {
    std::function<void(std::shared_ptr<Request>)> cb;
    {
      std::lock_guard<std::mutex> lk(cb_mu_);
      auto it = callbacks_.find(rsp->meta.message_id);
      if (it == callbacks_.end()) {
        SS_LOG_WARN("response for unknown message id %lld", (long long)rsp->meta.message_id);
        return;
      }
      cb = std::move(it->second);
      callbacks_.erase(it);
    }
    pool_->submit([cb, rsp] { cb(rsp); });
  }

  Addr addr_;
  int lfd_ = -1;
  int client_id_ = -3;
  std::atomic<bool> running_{false};
  std::atomic<int64_t> msg_counter_{0};
  std::unique_ptr<ThreadPool> pool_;
  std::thread accept_thread_;
  std::vector<std::thread> readers_;
  std::vector<int> in_fds_;
  mutable std::shared_mutex route_mu_, handler_mu_;
  mutable std::mutex cb_mu_, conn_mu_;
  std::map<int, Addr> route_;
  std::unordered_map<int32_t, Handler> handlers_;
  std::unordered_map<int64_t, std::function<void(std::shared_ptr<Request>)>> callbacks_;
  std::unordered_map<int, std::shared_ptr<Conn>> out_;
};

}  // namespace ss
