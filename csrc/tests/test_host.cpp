// test_host.cpp — native unit tests of the host runtime (no GPU), built plain
// and with -fsanitize=address,undefined and -fsanitize=thread by
// swiftsnails_amd/_build.py (build_cpp_tests) and run by tests/test_cpp.py.
//
// The reference's suite is a single gtest binary including every *_test.h
// (/root/reference/src/unitest/main.cpp:1-38) run under valgrind
// (unitest/valgrind.sh); gtest is not available here, so a ~40-line harness
// below registers TEST()s and runs them (optionally filtered by argv[1]).
// Coverage follows the reference's areas: codec, strings, config,
// channel/pool/barriers, router, table + text dump, the loopback transfer
// (transfer_test.h: send 2008 to yourself, reply 2009), plus the data loader.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "swiftsnails.h"  // the umbrella header: every host-runtime header

namespace {

struct Registry {
  std::vector<std::pair<std::string, std::function<void()>>> tests;
  static Registry& get() {
    static Registry r;
    return r;
  }
};
struct Reg {
  Reg(const char* n, std::function<void()> f) { Registry::get().tests.emplace_back(n, f); }
};
int g_fail = 0;

#define TEST(name)                              \
  static void test_##name();                    \
  static Reg reg_##name(#name, test_##name);    \
  static void test_##name()
#define EXPECT(cond)                                                                   \
  do {                                                                                 \
    if (!(cond)) {                                                                     \
      std::fprintf(stderr, "  EXPECT failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                                        \
    }                                                                                  \
  } while (0)

std::string tmpfile(const std::string& name, const std::string& body) {
  const char* d = std::getenv("TMPDIR");
  std::string p = std::string(d ? d : "/tmp") + "/ss_cpp_" + std::to_string(::getpid()) + "_" + name;
  std::ofstream(p) << body;
  return p;
}

}  // namespace

using namespace ss;

// ---------------------------------------------------------------- Vec
// (reference utils/vec1.h; its vec1_test.h only prints)
TEST(vec_arithmetic_codec_text) {
  Vec a{1, 2, 3}, b{4, 5, 6};
  EXPECT(a.dot(b) == 32);
  EXPECT((a + b) == (Vec{5, 7, 9}));
  EXPECT((b - a) == (Vec{3, 3, 3}));
  EXPECT((a * b) == (Vec{4, 10, 18}));
  EXPECT((b / a) == (Vec{4, 2.5, 2}));
  EXPECT((2.0 * a) == (Vec{2, 4, 6}));
  EXPECT((a * 2.0) == (Vec{2, 4, 6}));
  EXPECT((a + 1.0) == (Vec{2, 3, 4}));
  EXPECT((1.0 - a) == (Vec{0, -1, -2}));
  EXPECT((6.0 / a) == (Vec{6, 3, 2}));
  EXPECT(sqrt(Vec{4, 9}) == (Vec{2, 3}));
  Vec c = a;
  c.axpy(-0.5, b);
  EXPECT(c == (Vec{-1, -0.5, 0}));
  auto o = outer(Vec{1, 2}, Vec{3, 4, 5});
  EXPECT(o.size() == 2 && o[1] == (Vec{6, 8, 10}));
  bool threw = false;
  try {
    a += Vec{1, 2};
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw);
  // random init: word2vec convention, |x| <= 0.5 / size, deterministic by seed
  Vec r(64), r2(64);
  r.rand_init(0.5, 7);
  r2.rand_init(0.5, 7);
  EXPECT(r == r2);
  bool in_range = true;
  for (size_t i = 0; i < r.size(); ++i) in_range &= std::fabs(r[i]) <= 0.5 / 64;
  EXPECT(in_range);
  r.reset();
  EXPECT(r.size() == 64 && r.norm2() == 0);
  // codec + text round trips (checkpoint line value part)
  BinaryBuffer bb;
  bb << a << Vec{} << b;
  Vec x, y, z;
  bb >> x >> y >> z;
  EXPECT(x == a && y.empty() && z == b);
  EXPECT(Vec::parse(Vec{0.25, -3, 1e-3}.to_string()) == (Vec{0.25, -3, 1e-3}));
  std::ostringstream os;
  os << Vec{1, 2.5};
  EXPECT(os.str() == "1 2.5");
}

// ---------------------------------------------------------------- codec
struct Apple {  // user struct with its own codec (Buffer_test.h:47-62)
  int weight;
  double price;
};
TEST(binary_buffer_roundtrip_and_growth) {
  BinaryBuffer b;
  const size_t cap0 = b.capacity();
  b << (int32_t)7 << (int64_t)-3 << 2.5f << 1.25 << std::string("hello");
  Apple a{3, 9.5};
  b << a;
  for (int i = 0; i < 2000; ++i) b << (int32_t)i;  // grows past the 1024-B start
  EXPECT(b.capacity() >= cap0);
  int32_t i32;
  int64_t i64;
  float f;
  double d;
  std::string s;
  Apple a2{};
  b >> i32 >> i64 >> f >> d >> s >> a2;
  EXPECT(i32 == 7 && i64 == -3 && f == 2.5f && d == 1.25 && s == "hello");
  EXPECT(a2.weight == 3 && a2.price == 9.5);
  for (int i = 0; i < 2000; ++i) {
    int32_t v;
    b >> v;
    EXPECT(v == i);
  }
  EXPECT(b.read_finished());
  BinaryBuffer m(std::move(b));  // move keeps contents
  EXPECT(m.size() > 8000);
}

// ---------------------------------------------------------------- strings
TEST(string_utils) {
  EXPECT(trim("  a b \t\n") == "a b");
  auto v = split("a,b;;c", ",;");
  EXPECT(v.size() == 3 && v[0] == "a" && v[2] == "c");
  auto kv = key_value_split("ip: tcp://1:2", ":");
  EXPECT(kv.first == "ip" && trim(kv.second) == "tcp://1:2");
  EXPECT(headswith("import x", "import"));
  EXPECT(format_string("%d-%s", 5, "x") == "5-x");
  const std::string p = tmpfile("lines.txt", "l1\nl2\nl3\n");
  FILE* fp = std::fopen(p.c_str(), "r");
  LineFileReader r;
  int n = 0;
  while (r.getline(fp)) ++n;
  std::fclose(fp);
  EXPECT(n == 3);
  std::remove(p.c_str());
}

// ---------------------------------------------------------------- config
TEST(config_first_definition_wins_and_import) {
  const std::string base = tmpfile("base.conf", "thread_num: 4\nshared: base\n");
  const std::string top = tmpfile(
      "top.conf", "# comment\nip: tcp://127.0.0.1:8080\nthread_num: 12\nimport " + base + "\n");
  ConfigParser c(top);
  c.parse();
  EXPECT(c.get_config("ip").to_string() == "tcp://127.0.0.1:8080");
  EXPECT(c.get_config("thread_num").to_int32() == 12);  // first definition wins
  EXPECT(c.get_config("shared").to_string() == "base");
  EXPECT(!c.has("missing"));
  bool threw = false;
  try {
    c.get_config("missing");
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT(threw);
  std::remove(base.c_str());
  std::remove(top.c_str());
}

// ---------------------------------------------------------------- concurrency
TEST(channel_mpmc_close_drains) {
  Channel<int> ch(16);
  std::atomic<long> sum{0};
  std::vector<std::thread> cons;
  for (int c = 0; c < 3; ++c)
    cons.emplace_back([&] {
      int v;
      while (ch.pop(v)) sum += v;
    });
  std::vector<std::thread> prod;
  for (int p = 0; p < 4; ++p)
    prod.emplace_back([&, p] {
      for (int i = 1; i <= 1000; ++i) ch.push(i);
    });
  for (auto& t : prod) t.join();
  ch.close();  // queued items are still delivered (reference drops them)
  for (auto& t : cons) t.join();
  EXPECT(sum == 4L * 1000 * 1001 / 2);
}

TEST(thread_pool_async_exec_count) {
  ThreadPool pool(4);
  std::atomic<int> n{0};
  for (int r = 0; r < 10; ++r) pool.parallel_for(4, [&](int) { ++n; });
  EXPECT(n == 40);  // AsynExec_test.h: async_exec(4, task) x 10 -> 40
}

TEST(state_barrier_timeout_and_release) {
  StateBarrier b;
  EXPECT(!b.block_for(0.05));
  std::thread t([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    b.set_state_valid();
  });
  EXPECT(b.block_for(5.0));
  t.join();
}

// ---------------------------------------------------------------- router
TEST(hashfrag_matches_reference_formula) {
  HashFrag hf;
  hf.init(7, 100);
  for (uint64_t k = 0; k < 5000; ++k) {
    const int frag = (int)(fmix64(k) % 100);
    // fragment i -> node i/(frag_num/num_nodes)+1, clamped to [1, num_nodes]
    int node = frag / (100 / 7) + 1;
    if (node > 7) node = 7;
    EXPECT(hf.to_node_id(k) == node);
  }
  BinaryBuffer bb;
  hf.serialize(bb);
  HashFrag h2;
  h2.deserialize(bb);
  for (uint64_t k = 0; k < 100; ++k) EXPECT(h2.to_node_id(k) == hf.to_node_id(k));
}

// ---------------------------------------------------------------- table
TEST(host_table_pull_push_text_roundtrip) {
  InitParams ip{0, 0.f, 0.f, 1, -1};
  OptParams op{0, 0.5f, 0, 0, 1e-8f, 0.9f, 0.999f, 1, 1, 0.05f, 1, 1, 0};  // SGD
  HostTable t(3, 5, ip, op);
  std::vector<uint64_t> keys = {1, 2, 3, 1ull << 40, ~0ull - 1};
  std::vector<float> out(keys.size() * 3);
  t.pull(keys.data(), keys.size(), out.data());
  for (float v : out) EXPECT(v == 0.f);
  std::vector<float> g(keys.size() * 3, 1.f);
  std::vector<std::thread> th;  // concurrent pushes on striped shards
  for (int i = 0; i < 4; ++i) th.emplace_back([&] { t.push(keys.data(), keys.size(), g.data()); });
  for (auto& x : th) x.join();
  t.pull(keys.data(), keys.size(), out.data());
  for (float v : out) EXPECT(v == -2.f);  // 4 pushes x (-0.5)
  EXPECT(t.size() == keys.size());
  const std::string p = tmpfile("dump.txt", "");
  EXPECT(t.write_text(p) > 0);  // bytes written
  std::ifstream in(p);
  std::string line;
  int n = 0;
  while (std::getline(in, line)) {
    EXPECT(line.find('\t') != std::string::npos);  // key<TAB>value
    ++n;
  }
  EXPECT(n == (int)keys.size());
  HostTable t2(3, 2, ip, op);
  EXPECT(t2.load_text(p) == keys.size());
  std::vector<float> o2(out.size());
  t2.pull(keys.data(), keys.size(), o2.data());
  EXPECT(o2 == out);
  std::remove(p.c_str());
}

// user-defined access methods: the reference's PullAccessMethod::init_param
// and PushAccessMethod::apply_push_value (sparse_access_method.h:10-48)
TEST(host_table_user_access_methods) {
  InitParams ip{0, 0.f, 0.f, 1, -1};
  OptParams op{1, 0.1f, 0, 0, 1e-8f, 0.9f, 0.999f, 1, 1, 0.05f, 1, 1, 0};  // AdaGrad layout
  HostTable t(2, 3, ip, op);
  EXPECT(t.width() == 4);
  // init: w = key / 10, state = 7; apply: clipped step w -= clamp(g, -1, 1), state counts pushes
  t.set_access_methods(
      [](uint64_t key, float* row, int dim, int width) {
        for (int j = 0; j < dim; ++j) row[j] = (float)key / 10.f;
        for (int j = dim; j < width; ++j) row[j] = 7.f;
      },
      [](uint64_t, float* row, const float* g, int dim, int width) {
        for (int j = 0; j < dim; ++j) row[j] -= std::max(-1.f, std::min(1.f, g[j]));
        for (int j = dim; j < width; ++j) row[j] += 1.f;
      });
  std::vector<uint64_t> keys = {10, 20, 30};
  std::vector<float> out(6);
  t.pull(keys.data(), 3, out.data());
  EXPECT(out[0] == 1.f && out[3] == 2.f && out[5] == 3.f);
  std::vector<float> g = {5.f, 0.25f, -3.f, 0.5f, 0.f, 0.f};
  t.push(keys.data(), 3, g.data());
  t.pull(keys.data(), 3, out.data());
  EXPECT(out[0] == 0.f && out[1] == 0.75f && out[2] == 3.f && out[3] == 1.5f && out[4] == 3.f);
  std::vector<float> rows(12);
  std::vector<uint8_t> found(3);
  t.get_rows(keys.data(), 3, rows.data(), found.data());
  EXPECT(found[0] && rows[2] == 8.f && rows[3] == 8.f);  // 7 + one push
  // batch form (interpreted callers): whole push at once
  t.set_batch_apply([](const uint64_t*, size_t n, float* r, const float* gg) {
    for (size_t i = 0; i < n; ++i) r[i * 4] += 100.f * gg[i * 2];
  });
  std::vector<float> g2 = {1.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  t.push(keys.data(), 1, g2.data());
  t.pull(keys.data(), 1, out.data());
  EXPECT(out[0] == 100.f);
  // a key pushed twice in one call reaches the rule once, gradients summed
  std::vector<uint64_t> kd = {10, 10};
  std::vector<float> gd = {1.f, 0.f, 2.f, 0.f};
  t.push(kd.data(), 2, gd.data());
  t.pull(keys.data(), 1, out.data());
  EXPECT(out[0] == 400.f);
  // pushing a key never pulled creates it with the user init first
  std::vector<uint64_t> k4 = {40};
  std::vector<float> g4 = {0.f, 0.f};
  t.set_batch_apply(nullptr);
  t.push(k4.data(), 1, g4.data());
  t.pull(k4.data(), 1, out.data());
  EXPECT(out[0] == 4.f);
}

// ---------------------------------------------------------------- transfer
TEST(transfer_loopback_2008_2009) {
  Transfer tr;
  tr.listen("");
  tr.add_handler(1, [](std::shared_ptr<Request> req, Request& rsp) {
    int32_t v = 0;
    req->cont >> v;
    rsp.cont << (int32_t)(v + 1);
  });
  tr.service_start(2);
  tr.register_node(1, tr.addr());  // its own address as node 1
  StateBarrier done;
  int32_t got = 0;
  Request r;
  r.meta.message_class = 1;
  r.cont << (int32_t)2008;
  r.call_back_handler = [&](std::shared_ptr<Request> rsp) {
    rsp->cont >> got;
    done.set_state_valid();
  };
  tr.send(std::move(r), 1);
  EXPECT(done.block_for(10.0));
  EXPECT(got == 2009);
  tr.service_end();
}

// ---------------------------------------------------------------- cluster
// Master + 2 servers + 2 workers in one process (threads), the full protocol:
// registration with deferred replies, hashfrag fetch, pull (lookup-or-init),
// push (SGD apply), finish, terminate + final dump.
#include "cluster.h"
TEST(cluster_master_servers_workers_inprocess) {
  ConfigParser mc;
  mc.parse_string("listen_addr: tcp://127.0.0.1:0\nexpected_node_num: 4\nfrag_num: 50\n");
  Master master(mc);
  const std::string maddr = master.addr();
  const std::string dump = tmpfile("cl_final.txt", "");
  ConfigParser nc;
  nc.parse_string("master_addr: " + maddr + "\noptimizer: sgd\nlearning_rate: 0.5\n" +
                  "param_output: " + dump + "\ninit_timeout: 30\n");
  std::thread mt([&] { master.run(); });
  std::vector<std::unique_ptr<Server>> servers;
  for (int i = 0; i < 2; ++i) servers.emplace_back(new Server(nc, 2));
  std::vector<std::thread> st;
  for (auto& s : servers)
    st.emplace_back([&s] {
      s->connect();
      s->wait_terminate(60);
    });
  std::vector<std::vector<float>> res(2);
  std::vector<std::thread> wt;
  for (int w = 0; w < 2; ++w)
    wt.emplace_back([&, w] {
      WorkerClient c(nc);
      c.connect();
      std::vector<uint64_t> keys = {1, 2, 3, 1000, 77777, (1ull << 40) + 5};
      std::vector<float> v;
      EXPECT(c.pull(keys.data(), keys.size(), v) == 2);
      std::vector<float> g(keys.size() * 2, 1.f);
      for (int r = 0; r < 2; ++r) c.push(keys.data(), keys.size(), g.data(), 2);
      c.finish();
    });
  for (auto& t : wt) t.join();
  mt.join();
  for (auto& t : st) t.join();
  // 2 workers x 2 pushes x (-0.5 * 1) -> -2 everywhere; each server dumped its shard
  size_t total = 0;
  for (auto& s : servers) {
    total += s->table().size();
    std::vector<uint64_t> k;
    std::vector<float> rows;
    s->table().export_all(k, rows);
    for (size_t i = 0; i < k.size(); ++i) EXPECT(rows[i * s->table().width()] == -2.f);
    std::remove((dump + ".s" + std::to_string(s->client_id())).c_str());
  }
  EXPECT(total == 6);
  std::remove(dump.c_str());
}

// ---------------------------------------------------------------- data input
TEST(sparse_dataset_parse_and_fill) {
  const std::string p = tmpfile("a.svm", "1 3:0.5 7\n0 9:2\n-1\n1 1 2 3 4 5 6\n");
  SparseDataset ds(p, "libsvm", 3, 0, 1);
  EXPECT(ds.rows() == 4 && ds.nnz() == 9 && ds.max_nnz() == 6 && ds.has_values());
  std::vector<uint64_t> k(2 * 4);
  std::vector<float> v(2 * 4), l(2);
  const uint64_t nxt = ds.fill(3, 2, 4, k.data(), v.data(), l.data(), 2);
  EXPECT(nxt == 1);
  EXPECT(k[0] == 1 && k[3] == 4 && l[0] == 1.f);  // row 3 truncated to 4 keys
  EXPECT(k[4] == 3 && k[5] == 7 && k[6] == kDataEmptyKey && v[4] == 0.5f && v[5] == 1.f);
  std::remove(p.c_str());
}

int main(int argc, char** argv) {
  const std::string filt = argc > 1 ? argv[1] : "";
  int ran = 0;
  for (auto& t : Registry::get().tests) {
    if (!filt.empty() && t.first.find(filt) == std::string::npos) continue;
    const int before = g_fail;
    try {
      t.second();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "  exception: %s\n", e.what());
      ++g_fail;
    }
    std::printf("[%s] %s\n", g_fail == before ? " OK " : "FAIL", t.first.c_str());
    ++ran;
  }
  std::printf("%d tests, %d failed expectations\n", ran, g_fail);
  return g_fail ? 1 : 0;
}
