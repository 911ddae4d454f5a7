// cluster.h — master / server / worker protocol for host (CPU) clusters.
//
// Reference (call stacks §3.1-3.4):
//   MasterTransferInit  core/system/master/init.h:21-171
//   MasterTerminate     core/system/master/terminate.h:15-109
//   NodeTransferInit / NodeHashfragInit  core/system/node_init.h:16-152
//   ServerInitPull/PushMethod  core/system/server/init.h:27-163
//   ServerTerminate     core/system/server/terminate.h:16-54
//   ClientTerminate     core/system/worker/terminate.h:17-58
//   GlobalPull/PushAccess      core/parameter/global_{pull,push}_access.h
//   ServerWorkerRoute   core/system/ServerWorkerRoute.h:14-84
//
// Protocol kept: ids (master 0, servers 1..S, workers INT_MAX-1, -2, ...),
// deferred registration replies carrying the whole route, hashfrag fetch from
// the master, pull = lookup-or-init, push = apply with periodic text backups
// every `param_backup_period` push requests, worker finish -> master tells
// every server to terminate -> servers dump the final table.
// Changes: payloads are SoA ([n][keys][rows], no per-key Val echo on pull
// requests), servers register their handlers BEFORE announcing themselves (no
// 3 s / 5 s sleeps needed), pull/push with no keys return immediately, and
// every wait has a timeout that raises instead of aborting the process.
#pragma once
#include <climits>
#include <memory>
#include <string>
#include <vector>

#include "config.h"
#include "hashfrag.h"
#include "host_table.h"
#include "transfer.h"

namespace ss {

struct RouteTable {
  std::vector<int> server_ids;
  std::vector<int> worker_ids;
  std::map<int, Addr> addrs;  // includes the master (id 0)
  void serialize(BinaryBuffer& bb) const {
    bb << (int32_t)(server_ids.size() + 1) << (int32_t)worker_ids.size();
    bb << (int32_t)addrs.size();
    for (auto& kv : addrs) bb << (int32_t)kv.first << kv.second.to_string();
    for (int s : server_ids) bb << (int32_t)s;
    for (int w : worker_ids) bb << (int32_t)w;
  }
  void deserialize(BinaryBuffer& bb) {
    int32_t ns = 0, nw = 0, na = 0;
    bb >> ns >> nw >> na;
    addrs.clear();
    for (int i = 0; i < na; ++i) {
      int32_t id;
      std::string a;
      bb >> id >> a;
      addrs[id] = Addr::parse(a);
    }
    server_ids.resize((size_t)(ns - 1));
    worker_ids.resize((size_t)nw);
    for (auto& s : server_ids) {
      int32_t v;
      bb >> v;
      s = v;
    }
    for (auto& w : worker_ids) {
      int32_t v;
      bb >> v;
      w = v;
    }
  }
};

inline InitParams init_from_config(const ConfigParser& c) {
  const std::string k = c.get("param_init", "zero");
  InitParams ip{kInitZero, 0.f, 0.f, 2015, -1};
  ip.kind = k == "uniform" ? kInitUniform : (k == "normal" ? kInitNormal : kInitZero);
  ip.scale = std::stof(c.get("param_init_scale", "0"));
  ip.state_init = std::stof(c.get("optimizer_state_init", "0"));
  ip.seed = std::stoull(c.get("param_init_seed", "2015"));
  return ip;
}
inline OptParams opt_from_config(const ConfigParser& c) {
  const std::string k = c.get("optimizer", "sgd");
  OptParams op{};
  op.kind = k == "adagrad" ? kOptAdaGrad : k == "ftrl" ? kOptFTRL : k == "adam" ? kOptAdam : kOptSGD;
  op.lr = std::stof(c.get("learning_rate", "0.01"));
  op.l1 = std::stof(c.get("l1", "0"));
  op.l2 = std::stof(c.get("l2", "0"));
  op.eps = std::stof(c.get("adagrad_eps", "1e-8"));
  op.beta1 = 0.9f;
  op.beta2 = 0.999f;
  op.bc1 = op.bc2 = 1.f;
  op.ftrl_alpha = std::stof(c.get("ftrl_alpha", "0.05"));
  op.ftrl_beta = std::stof(c.get("ftrl_beta", "1"));
  op.grad_scale = 1.f;
  op.clip = 0.f;
  return op;
}

// ===================================================================== master
class Master : NonCopyable {
 public:
  explicit Master(const ConfigParser& cfg) : cfg_(cfg) {
    expected_ = cfg.get_config("expected_node_num").to_int32();
    timeout_ = std::stod(cfg.get("master_time_out", "60"));
    frag_num_ = std::stoi(cfg.get("frag_num", "1000"));
    tr_.listen(cfg.get("listen_addr", ""));
    tr_.set_client_id(0);
    tr_.register_node(0, tr_.addr());
    tr_.add_handler(NODE_INIT_ADDRESS, [this](std::shared_ptr<Request> req, Request&) {
      int32_t is_server = 0;
      std::string a;
      req->cont >> is_server >> a;
      std::lock_guard<std::mutex> lk(mu_);
      int id = is_server ? (int)route_.server_ids.size() + 1
                         : INT_MAX - 1 - (int)route_.worker_ids.size();
      (is_server ? route_.server_ids : route_.worker_ids).push_back(id);
      route_.addrs[id] = Addr::parse(a);
      tr_.register_node(id, Addr::parse(a));
      pending_.push_back({id, req->meta.message_id});  // deferred reply
      if ((int)pending_.size() == expected_) registered_.set_state_valid();
    });
    tr_.add_handler(NODE_ASKFOR_HASHFRAG, [this](std::shared_ptr<Request>, Request& rsp) {
      hashfrag_ready_.block();
      frag_.serialize(rsp.cont);
    });
    tr_.add_handler(WORKER_FINISH_WORK, [this](std::shared_ptr<Request>, Request& rsp) {
      rsp.cont << (int32_t)1;
      if (++finished_ == (int)route_.worker_ids.size()) all_finished_.set_state_valid();
    });
    tr_.service_start(std::stoi(cfg.get("async_exec_num", "4")));
  }
  ~Master() { tr_.service_end(); }

  std::string addr() const { return tr_.addr().to_string(); }

  // registration: returns once every node has its route and the hashfrag
  void init() {
    if (!registered_.block_for(timeout_))
      throw Error("master: node registration timed out (" + std::to_string(pending_.size()) + "/" +
                  std::to_string(expected_) + ")");
    std::lock_guard<std::mutex> lk(mu_);
    SS_CHECK_MSG(!route_.server_ids.empty(), "no server registered");
    frag_.init((int)route_.server_ids.size(), frag_num_);
    hashfrag_ready_.set_state_valid();
    route_.addrs[0] = tr_.addr();
    for (auto& p : pending_) {  // send_route_to_workers (master/init.h:74-99)
      Request rsp;
      route_.serialize(rsp.cont);
      rsp.meta.message_id = p.second;
      rsp.meta.client_id = p.first;  // the node learns its id from the reply
      tr_.send_response(std::move(rsp), p.first);
    }
  }

  // wait for every worker to finish, then terminate every server
  void terminate() {
    if (!route_.worker_ids.empty() && !all_finished_.block_for(1e9))
      throw Error("master: workers did not finish");
    CountDownLatch acks((long)route_.server_ids.size());
    for (int s : route_.server_ids) {
      Request r;
      r.meta.message_class = SERVER_TOLD_TO_TERMINATE;
      r.call_back_handler = [&acks](std::shared_ptr<Request>) { acks.count_down(); };
      tr_.send(std::move(r), s);
    }
    if (!acks.wait_for(timeout_)) throw Error("master: servers did not acknowledge terminate");
    SS_LOG_INFO("Master terminated normally!");
  }
  void run() {
    init();
    terminate();
  }
  int server_num() const { return (int)route_.server_ids.size(); }
  int worker_num() const { return (int)route_.worker_ids.size(); }

 private:
  const ConfigParser& cfg_;
  Transfer tr_;
  int expected_ = 0, frag_num_ = 1000;
  double timeout_ = 60;
  std::mutex mu_;
  RouteTable route_;
  std::vector<std::pair<int, int64_t>> pending_;
  StateBarrier registered_, hashfrag_ready_, all_finished_;
  std::atomic<int> finished_{0};
  HashFrag frag_;
};

// ======================================================================= node
// Common node bring-up (NodeTransferInit + NodeHashfragInit).
class Node : NonCopyable {
 public:
  Node(const ConfigParser& cfg, bool is_server) : cfg_(cfg), is_server_(is_server) {
    timeout_ = std::stod(cfg.get("init_timeout", "60"));
    tr_.listen(cfg.get("node_listen_addr", ""));
  }
  virtual ~Node() { tr_.service_end(); }

  void connect() {
    tr_.service_start(std::stoi(cfg_.get("async_exec_num", "4")));
    tr_.register_node(0, Addr::parse(cfg_.get_config("master_addr").to_string()));
    StateBarrier b;
    Request r;
    r.meta.message_class = NODE_INIT_ADDRESS;
    is_server_ ? r.set_server() : r.set_worker();
    r.cont << (int32_t)(is_server_ ? 1 : 0) << tr_.addr().to_string();
    r.call_back_handler = [this, &b](std::shared_ptr<Request> rsp) {
      route_.deserialize(rsp->cont);
      for (auto& kv : route_.addrs)
        if (kv.first != 0) tr_.register_node(kv.first, kv.second);
      tr_.set_client_id(rsp->meta.client_id);
      b.set_state_valid();
    };
    tr_.send(std::move(r), 0);
    if (!b.block_for(timeout_)) throw Error("node: registration with master timed out");
    StateBarrier hb;
    Request h;
    h.meta.message_class = NODE_ASKFOR_HASHFRAG;
    h.call_back_handler = [this, &hb](std::shared_ptr<Request> rsp) {
      frag_.deserialize(rsp->cont);
      hb.set_state_valid();
    };
    tr_.send(std::move(h), 0);
    if (!hb.block_for(timeout_)) throw Error("node: hashfrag fetch timed out");
  }
  int client_id() const { return tr_.client_id(); }
  const HashFrag& hashfrag() const { return frag_; }
  const RouteTable& route() const { return route_; }
  Transfer& transfer() { return tr_; }

 protected:
  const ConfigParser& cfg_;
  bool is_server_;
  double timeout_ = 60;
  Transfer tr_;
  RouteTable route_;
  HashFrag frag_;
};

// ===================================================================== server
class Server : public Node {
 public:
  Server(const ConfigParser& cfg, int dim) : Node(cfg, true) {
    table_.reset(new HostTable(dim, std::stoi(cfg.get("shard_num", "8")), init_from_config(cfg),
                               opt_from_config(cfg)));
    backup_period_ = std::stoi(cfg.get("param_backup_period", "0"));
    backup_root_ = cfg.get("param_backup_root", ".");
    output_ = cfg.get("param_output", "-");
    // handlers first, then announce (no race with early worker requests)
    tr_.add_handler(WORKER_PULL_REQUEST, [this](std::shared_ptr<Request> req, Request& rsp) {
      uint32_t n = 0;
      req->cont >> n;
      std::vector<uint64_t> keys(n);
      req->cont.get_raw(keys.data(), n * 8ull);
      std::vector<float> vals((size_t)n * table_->dim());
      table_->pull(keys.data(), n, vals.data());
      rsp.cont << n << (uint32_t)table_->dim();
      rsp.cont.put_raw(vals.data(), vals.size() * 4);
    });
    tr_.add_handler(WORKER_PUSH_REQUEST, [this](std::shared_ptr<Request> req, Request& rsp) {
      uint32_t n = 0, d = 0;
      req->cont >> n >> d;
      SS_CHECK_MSG((int)d == table_->dim(), "push dim mismatch");
      std::vector<uint64_t> keys(n);
      std::vector<float> g((size_t)n * d);
      req->cont.get_raw(keys.data(), n * 8ull);
      req->cont.get_raw(g.data(), g.size() * 4);
      table_->push(keys.data(), n, g.data());
      rsp.cont << (int32_t)1234;
      const int c = ++push_counter_;
      if (backup_period_ > 0 && c % backup_period_ == 0) backup(c);
    });
    tr_.add_handler(SERVER_TOLD_TO_TERMINATE, [this](std::shared_ptr<Request>, Request& rsp) {
      if (!output_.empty()) table_->write_text(shard_path(output_));
      rsp.cont << (int32_t)1;
      terminated_.set_state_valid();
    });
  }
  // blocks until the master tells this server to terminate
  void wait_terminate(double timeout_s = 1e9) {
    if (!terminated_.block_for(timeout_s)) throw Error("server: terminate wait timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));  // let the ack flush
  }
  HostTable& table() { return *table_; }
  int push_count() const { return push_counter_.load(); }
  std::string backup(int c) {
    const std::string path = shard_path(backup_root_ + "/param-" + std::to_string(c) + ".txt");
    table_->write_text(path);
    return path;
  }
  // With several servers every one writes its own shard file (`<path>.s<id>`;
  // the reference's servers each dumped to their own reducer stdout); a single
  // server and "-" (stdout) keep the plain name.
  std::string shard_path(const std::string& path) const {
    if (path == "-" || route_.server_ids.size() <= 1) return path;
    return path + ".s" + std::to_string(client_id());
  }

 private:
  std::unique_ptr<HostTable> table_;
  int backup_period_ = 0;
  std::string backup_root_, output_;
  std::atomic<int> push_counter_{0};
  StateBarrier terminated_;
};

// ===================================================================== worker
class WorkerClient : public Node {
 public:
  explicit WorkerClient(const ConfigParser& cfg) : Node(cfg, false) {
    req_timeout_ = std::stod(cfg.get("request_timeout", "600"));
  }

  // pull_with_barrier: out[n * dim] in key order; returns dim
  int pull(const uint64_t* keys, size_t n, std::vector<float>& out) {
    if (n == 0) return 0;  // (reference blocks forever on an empty set)
    std::map<int, std::vector<uint32_t>> by_node;
    for (size_t i = 0; i < n; ++i) by_node[frag_.to_node_id(keys[i])].push_back((uint32_t)i);
    CountDownLatch latch((long)by_node.size());
    std::atomic<int> dim{0};
    std::mutex mu;
    for (auto& kv : by_node) {
      Request r;
      r.meta.message_class = WORKER_PULL_REQUEST;
      r.set_worker();
      auto& idx = kv.second;
      r.cont << (uint32_t)idx.size();
      for (uint32_t i : idx) r.cont << keys[i];
      const std::vector<uint32_t>* pidx = &idx;
      r.call_back_handler = [&, pidx](std::shared_ptr<Request> rsp) {
        uint32_t m = 0, d = 0;
        rsp->cont >> m >> d;
        {
          std::lock_guard<std::mutex> lk(mu);
          if (out.size() < n * d) out.resize(n * d);
          dim = (int)d;
          const float* v = reinterpret_cast<const float*>(rsp->cont.data() + rsp->cont.cursor());
          for (uint32_t j = 0; j < m; ++j)
            std::copy(v + (size_t)j * d, v + (size_t)(j + 1) * d, out.data() + (size_t)(*pidx)[j] * d);
        }
        latch.count_down();
      };
      tr_.send(std::move(r), kv.first);
    }
    if (!latch.wait_for(req_timeout_)) throw Error("pull timed out");
    return dim.load();
  }

  // push_with_barrier: grads[n * dim]; duplicate keys are merged by the server
  void push(const uint64_t* keys, size_t n, const float* grads, int dim) {
    if (n == 0) return;
    std::map<int, std::vector<uint32_t>> by_node;
    for (size_t i = 0; i < n; ++i) by_node[frag_.to_node_id(keys[i])].push_back((uint32_t)i);
    CountDownLatch latch((long)by_node.size());
    for (auto& kv : by_node) {
      Request r;
      r.meta.message_class = WORKER_PUSH_REQUEST;
      r.set_worker();
      r.cont << (uint32_t)kv.second.size() << (uint32_t)dim;
      for (uint32_t i : kv.second) r.cont << keys[i];
      for (uint32_t i : kv.second) r.cont.put_raw(grads + (size_t)i * dim, (size_t)dim * 4);
      r.call_back_handler = [&latch](std::shared_ptr<Request>) { latch.count_down(); };
      tr_.send(std::move(r), kv.first);
    }
    if (!latch.wait_for(req_timeout_)) throw Error("push timed out");
  }

  // ClientTerminate (worker/terminate.h:37-51), without the 5 s sleep
  void finish() {
    StateBarrier b;
    Request r;
    r.meta.message_class = WORKER_FINISH_WORK;
    r.call_back_handler = [&b](std::shared_ptr<Request>) { b.set_state_valid(); };
    tr_.send(std::move(r), 0);
    if (!b.block_for(timeout_)) throw Error("worker: finish ack timed out");
  }

 private:
  double req_timeout_ = 600;
};

}  // namespace ss
