// module.cpp — pybind11 module `_ss_host`: the host C++ runtime.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "buffer.h"
#include "channel.h"
#include "cluster.h"
#include "config.h"
#include "dataio.h"
#include "hashfrag.h"
#include "host_table.h"
#include "ss/a2a_schedule.h"
#include "ss/hash.h"
#include "string_util.h"
#include "transfer.h"

namespace py = pybind11;
using namespace ss;

using u64arr = py::array_t<uint64_t, py::array::c_style | py::array::forcecast>;
using f32arr = py::array_t<float, py::array::c_style | py::array::forcecast>;

static InitParams mk_init(int kind, float scale, float state_init, uint64_t seed, int zero_bit) {
  return InitParams{kind, scale, state_init, seed, zero_bit};
}
static OptParams mk_opt(int kind, float lr, float l1, float l2, float eps, float beta1, float beta2,
                        float bc1, float bc2, float alpha, float beta, float grad_scale,
                        float clip) {
  return OptParams{kind, lr, l1, l2, eps, beta1, beta2, bc1, bc2, alpha, beta, grad_scale, clip};
}

PYBIND11_MODULE(_ss_host, m) {
  m.doc() = "SwiftSnails-AMD host runtime (config, codec, router, CPU table, TCP RPC, cluster)";
  py::register_exception<Error>(m, "SSError", PyExc_RuntimeError);

  // ---- hashing
  m.def("fmix64", &fmix64);
  m.def("fmix64_array", [](u64arr a) {
    auto r = a.unchecked<1>();
    py::array_t<uint64_t> out(r.shape(0));
    auto o = out.mutable_unchecked<1>();
    for (py::ssize_t i = 0; i < r.shape(0); ++i) o(i) = fmix64(r(i));
    return out;
  });

  // ---- alltoallv peer schedule (the RCCL communicator's, csrc/hip/comm.cpp)
  m.def("a2a_schedule",
        [](int rank, int nranks, std::vector<long long> sc, std::vector<long long> sd,
           std::vector<long long> rc, std::vector<long long> rd, int eb, long long send_cap,
           long long recv_cap) {
          py::list out;
          try {
            for (const A2aStep& x : a2a_schedule(rank, nranks, sc, sd, rc, rd, eb, send_cap,
                                                 recv_cap))
              out.append(py::make_tuple(x.k, x.to, x.send_off, x.send_bytes, x.from, x.recv_off,
                                        x.recv_bytes));
          } catch (const std::invalid_argument& e) {
            throw py::value_error(e.what());
          }
          return out;
        },
        py::arg("rank"), py::arg("nranks"), py::arg("scounts"), py::arg("sdispls"),
        py::arg("rcounts"), py::arg("rdispls"), py::arg("elem_bytes"), py::arg("send_cap") = -1,
        py::arg("recv_cap") = -1);

  // ---- strings
  m.def("trim", &trim);
  m.def("split", &split);
  m.def("key_value_split", &key_value_split);
  m.def("startswith", &startswith);

  // ---- config
  py::class_<ConfigParser>(m, "ConfigParser", py::module_local())
      .def(py::init<>())
      .def(py::init<std::string>())
      .def("load_conf", &ConfigParser::load_conf)
      .def("parse", &ConfigParser::parse)
      .def("parse_file", py::overload_cast<const std::string&>(&ConfigParser::parse_file))
      .def("parse_string", &ConfigParser::parse_string, py::arg("text"), py::arg("base_dir") = ".")
      .def("clear", &ConfigParser::clear)
      .def("has", &ConfigParser::has)
      .def("get", &ConfigParser::get)
      .def("get_config", [](const ConfigParser& c, const std::string& k) { return c.get_config(k).value; })
      .def("get_int32", [](const ConfigParser& c, const std::string& k) { return c.get_config(k).to_int32(); })
      .def("get_int64", [](const ConfigParser& c, const std::string& k) { return c.get_config(k).to_int64(); })
      .def("get_float", [](const ConfigParser& c, const std::string& k) { return c.get_config(k).to_float(); })
      .def("get_bool", [](const ConfigParser& c, const std::string& k) { return c.get_config(k).to_bool(); })
      .def("register_config", &ConfigParser::register_config, py::arg("key"), py::arg("value") = "")
      .def("set", &ConfigParser::set)
      .def("erase", &ConfigParser::erase)
      .def("items", &ConfigParser::items)
      .def("dump", &ConfigParser::dump)
      .def("__len__", &ConfigParser::size);
  m.def("global_config", &global_config, py::return_value_policy::reference);

  // ---- binary codec
  py::class_<BinaryBuffer>(m, "BinaryBuffer", py::module_local())
      .def(py::init<>())
      .def(py::init([](py::bytes b) { return BinaryBuffer(std::string(b)); }))
      .def("put_i32", [](BinaryBuffer& b, int32_t v) { b << v; })
      .def("put_i64", [](BinaryBuffer& b, int64_t v) { b << v; })
      .def("put_u64", [](BinaryBuffer& b, uint64_t v) { b << v; })
      .def("put_f32", [](BinaryBuffer& b, float v) { b << v; })
      .def("put_f64", [](BinaryBuffer& b, double v) { b << v; })
      .def("put_str", [](BinaryBuffer& b, const std::string& v) { b << v; })
      .def("get_i32", [](BinaryBuffer& b) { int32_t v; b >> v; return v; })
      .def("get_i64", [](BinaryBuffer& b) { int64_t v; b >> v; return v; })
      .def("get_u64", [](BinaryBuffer& b) { uint64_t v; b >> v; return v; })
      .def("get_f32", [](BinaryBuffer& b) { float v; b >> v; return v; })
      .def("get_f64", [](BinaryBuffer& b) { double v; b >> v; return v; })
      .def("get_str", [](BinaryBuffer& b) { std::string v; b >> v; return v; })
      .def("read_finished", &BinaryBuffer::read_finished)
      .def("size", &BinaryBuffer::size)
      .def("capacity", &BinaryBuffer::capacity)
      .def("cursor", &BinaryBuffer::cursor)
      .def("clear", &BinaryBuffer::clear)
      .def("bytes", [](const BinaryBuffer& b) { return py::bytes(b.str()); });

  // ---- router
  py::class_<HashFrag>(m, "HashFrag", py::module_local())
      .def(py::init<>())
      .def(py::init<int, int>())
      .def("init", &HashFrag::init)
      .def("to_node_id", &HashFrag::to_node_id)
      .def("to_node_ids", [](const HashFrag& h, u64arr k) {
        auto r = k.unchecked<1>();
        py::array_t<int32_t> out(r.shape(0));
        auto o = out.mutable_unchecked<1>();
        for (py::ssize_t i = 0; i < r.shape(0); ++i) o(i) = h.to_node_id(r(i));
        return out;
      })
      .def("serialize", [](const HashFrag& h) { BinaryBuffer b; h.serialize(b); return py::bytes(b.str()); })
      .def("deserialize", [](HashFrag& h, py::bytes d) { BinaryBuffer b{std::string(d)}; h.deserialize(b); })
      .def("map_table", &HashFrag::map_table)
      .def_property_readonly("num_nodes", &HashFrag::num_nodes)
      .def_property_readonly("num_frags", &HashFrag::num_frags);

  // ---- optimizer params (shared layout with the device module)
  py::class_<InitParams>(m, "InitParams", py::module_local())
      .def(py::init(&mk_init), py::arg("kind") = 0, py::arg("scale") = 0.f,
           py::arg("state_init") = 0.f, py::arg("seed") = 0, py::arg("zero_bit") = -1);
  py::class_<OptParams>(m, "OptParams", py::module_local())
      .def(py::init(&mk_opt), py::arg("kind") = 1, py::arg("lr") = 0.05f, py::arg("l1") = 0.f,
           py::arg("l2") = 0.f, py::arg("eps") = 1e-8f, py::arg("beta1") = 0.9f,
           py::arg("beta2") = 0.999f, py::arg("bc1") = 1.f, py::arg("bc2") = 1.f,
           py::arg("alpha") = 0.05f, py::arg("beta") = 1.f, py::arg("grad_scale") = 1.f,
           py::arg("clip") = 0.f);

  // ---- CPU table
  py::class_<HostTable>(m, "HostTable", py::module_local())
      .def(py::init<int, int, InitParams, OptParams, int, size_t>(), py::arg("dim"),
           py::arg("shard_num"), py::arg("init"), py::arg("opt"), py::arg("nthreads") = 0,
           py::arg("cap_per_shard") = 1024)
      .def_property_readonly("dim", &HostTable::dim)
      .def_property_readonly("width", &HostTable::width)
      .def_property_readonly("shard_num", &HostTable::shard_num)
      .def("to_shard_id", &HostTable::to_shard_id)
      .def("set_opt", &HostTable::set_opt)
      .def("size", &HostTable::size)
      .def("pull", [](HostTable& t, u64arr k) {
        py::array_t<float> out({(py::ssize_t)k.size(), (py::ssize_t)t.dim()});
        {
          py::gil_scoped_release g;
          t.pull(k.data(), (size_t)k.size(), out.mutable_data());
        }
        return out;
      })
      .def("push", [](HostTable& t, u64arr k, f32arr g) {
        SS_CHECK_MSG((size_t)g.size() == (size_t)k.size() * t.dim(), "grads must be [n, dim]");
        py::gil_scoped_release rel;
        t.push(k.data(), (size_t)k.size(), g.data());
      })
      .def("assign", [](HostTable& t, u64arr k, f32arr r) {
        SS_CHECK_MSG((size_t)r.size() == (size_t)k.size() * t.width(), "rows must be [n, width]");
        py::gil_scoped_release rel;
        t.assign(k.data(), (size_t)k.size(), r.data());
      })
      .def("set_batch_apply", [](HostTable& t, py::object fn) {
        // fn(keys u64[n], rows f32[n, width], grads f32[n, dim]) -> new rows
        if (fn.is_none()) {
          t.set_batch_apply(nullptr);
          return;
        }
        auto f = std::make_shared<py::object>(fn);
        const int dim = t.dim(), width = t.width();
        t.set_batch_apply([f, dim, width](const uint64_t* keys, size_t n, float* rows,
                                          const float* grads) {
          py::gil_scoped_acquire gil;
          py::array_t<uint64_t> ka((py::ssize_t)n);
          std::memcpy(ka.mutable_data(), keys, n * 8);
          py::array_t<float> ra({(py::ssize_t)n, (py::ssize_t)width});
          std::memcpy(ra.mutable_data(), rows, n * (size_t)width * 4);
          py::array_t<float> ga({(py::ssize_t)n, (py::ssize_t)dim});
          std::memcpy(ga.mutable_data(), grads, n * (size_t)dim * 4);
          auto out = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(
              (*f)(ka, ra, ga));
          SS_CHECK_MSG(out && (size_t)out.size() == n * (size_t)width,
                       "push method must return rows of shape [n, width]");
          std::memcpy(rows, out.data(), n * (size_t)width * 4);
        });
      }, py::arg("fn"))
      .def("get_rows", [](HostTable& t, u64arr k) {
        py::array_t<float> rows({(py::ssize_t)k.size(), (py::ssize_t)t.width()});
        py::array_t<uint8_t> found((py::ssize_t)k.size());
        t.get_rows(k.data(), (size_t)k.size(), rows.mutable_data(), found.mutable_data());
        return py::make_tuple(rows, found);
      })
      .def("export", [](HostTable& t) {
        std::vector<uint64_t> k;
        std::vector<float> r;
        t.export_all(k, r);
        py::array_t<uint64_t> ka((py::ssize_t)k.size());
        std::memcpy(ka.mutable_data(), k.data(), k.size() * 8);
        py::array_t<float> ra({(py::ssize_t)k.size(), (py::ssize_t)t.width()});
        if (!r.empty()) std::memcpy(ra.mutable_data(), r.data(), r.size() * 4);
        return py::make_tuple(ka, ra);
      })
      .def("write_text", &HostTable::write_text, py::arg("path"), py::arg("precision") = 9,
           py::arg("with_state") = false, py::call_guard<py::gil_scoped_release>())
      .def("load_text", &HostTable::load_text, py::call_guard<py::gil_scoped_release>());

  // ---- text checkpoint codec (host half of K8)
  m.def("format_rows", [](u64arr keys, f32arr rows, int dim, int width, bool with_state,
                          int precision, int nthreads) {
    SS_CHECK_MSG((size_t)rows.size() == (size_t)keys.size() * width, "rows must be [n, width]");
    std::string s;
    {
      py::gil_scoped_release rel;
      s = format_rows(keys.data(), rows.data(), (size_t)keys.size(), dim, width, with_state,
                      precision, nthreads);
    }
    return py::bytes(s);
  }, py::arg("keys"), py::arg("rows"), py::arg("dim"), py::arg("width"),
     py::arg("with_state") = false, py::arg("precision") = 9, py::arg("nthreads") = 8);
  m.def("parse_rows", [](py::bytes data, int dim, int width, float state_init, int nthreads) {
    std::string buf = data;
    std::vector<std::pair<size_t, size_t>> chunks;
    {
      const size_t n = buf.size();
      const size_t per = std::max<size_t>(1, n / (size_t)std::max(1, nthreads));
      size_t a = 0;
      while (a < n) {
        size_t b = std::min(n, a + per);
        while (b < n && buf[b - 1] != '\n') ++b;
        chunks.push_back({a, b});
        a = b;
      }
    }
    std::vector<std::vector<uint64_t>> ks(chunks.size());
    std::vector<std::vector<float>> rs(chunks.size());
    std::vector<int> bad(chunks.size(), 0);
    {
      py::gil_scoped_release rel;
      std::vector<std::thread> th;
      for (size_t c = 0; c < chunks.size(); ++c)
        th.emplace_back([&, c] {
          size_t p = chunks[c].first;
          std::vector<float> row((size_t)width);
          while (p < chunks[c].second) {
            size_t e = buf.find('\n', p);
            if (e == std::string::npos || e > chunks[c].second) e = chunks[c].second;
            if (e > p) {
              std::string line = buf.substr(p, e - p);
              for (int j = 0; j < width; ++j) row[j] = j < dim ? 0.f : state_init;
              uint64_t k;
              if (parse_row_line(line.c_str(), dim, width, &k, row.data())) {
                ks[c].push_back(k);
                rs[c].insert(rs[c].end(), row.begin(), row.end());
              } else {
                bad[c]++;
              }
            }
            p = e + 1;
          }
        });
      for (auto& t : th) t.join();
    }
    size_t n = 0;
    for (auto& k : ks) n += k.size();
    for (int b : bad) SS_CHECK_MSG(b == 0, "malformed checkpoint line(s)");
    py::array_t<uint64_t> ka((py::ssize_t)n);
    py::array_t<float> ra({(py::ssize_t)n, (py::ssize_t)width});
    size_t o = 0;
    for (size_t c = 0; c < ks.size(); ++c) {
      std::memcpy(ka.mutable_data() + o, ks[c].data(), ks[c].size() * 8);
      std::memcpy(ra.mutable_data() + o * width, rs[c].data(), rs[c].size() * 4);
      o += ks[c].size();
    }
    return py::make_tuple(ka, ra);
  }, py::arg("data"), py::arg("dim"), py::arg("width"), py::arg("state_init") = 0.f,
     py::arg("nthreads") = 8);

  // ---- TCP RPC
  py::class_<Request, std::shared_ptr<Request>>(m, "Request")
      .def(py::init<>())
      .def_property("message_class", [](const Request& r) { return r.meta.message_class; },
                    [](Request& r, int v) { r.meta.message_class = v; })
      .def_property_readonly("message_id", [](const Request& r) { return r.meta.message_id; })
      .def_property_readonly("client_id", [](const Request& r) { return r.meta.client_id; })
      .def("is_response", &Request::is_response)
      .def_property("payload", [](const Request& r) { return py::bytes(r.cont.str()); },
                    [](Request& r, py::bytes b) { r.cont = BinaryBuffer(std::string(b)); });
  py::class_<Transfer>(m, "Transfer", py::module_local())
      .def(py::init<>())
      .def("listen", &Transfer::listen, py::arg("addr") = "")
      .def("service_start", &Transfer::service_start, py::arg("async_threads") = 4)
      .def("service_end", &Transfer::service_end, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("addr", [](const Transfer& t) { return t.addr().to_string(); })
      .def_property("client_id", &Transfer::client_id, &Transfer::set_client_id)
      .def("register_node", [](Transfer& t, int id, const std::string& a) { t.register_node(id, Addr::parse(a)); })
      .def("delete_node", &Transfer::delete_node)
      .def("has_node", &Transfer::has_node)
      .def("pending_callbacks", &Transfer::pending_callbacks)
      .def("add_handler", [](Transfer& t, int cls, std::function<py::bytes(py::bytes)> fn) {
        // Python handler: payload bytes -> response bytes (b"" = deferred reply)
        t.add_handler(cls, [fn](std::shared_ptr<Request> req, Request& rsp) {
          py::gil_scoped_acquire g;
          std::string out = fn(py::bytes(req->cont.str()));
          rsp.cont = BinaryBuffer(out);
        });
      })
      .def("send", [](Transfer& t, int cls, py::bytes payload, int to,
                      std::function<void(py::bytes)> cb) {
        Request r;
        r.meta.message_class = cls;
        r.cont = BinaryBuffer(std::string(payload));
        if (cb)
          r.call_back_handler = [cb](std::shared_ptr<Request> rsp) {
            py::gil_scoped_acquire g;
            cb(py::bytes(rsp->cont.str()));
          };
        py::gil_scoped_release rel;
        return t.send(std::move(r), to);
      }, py::arg("message_class"), py::arg("payload"), py::arg("to"), py::arg("callback") = nullptr)
      .def("call", [](Transfer& t, int cls, py::bytes payload, int to, double timeout) {
        // synchronous request/response helper
        auto res = std::make_shared<std::string>();
        auto bar = std::make_shared<StateBarrier>();
        Request r;
        r.meta.message_class = cls;
        r.cont = BinaryBuffer(std::string(payload));
        r.call_back_handler = [res, bar](std::shared_ptr<Request> rsp) {
          *res = rsp->cont.str();
          bar->set_state_valid();
        };
        {
          py::gil_scoped_release rel;
          t.send(std::move(r), to);
          if (!bar->block_for(timeout)) throw Error("call timed out");
        }
        return py::bytes(*res);
      }, py::arg("message_class"), py::arg("payload"), py::arg("to"), py::arg("timeout") = 30.0);
  m.def("get_local_ip", &get_local_ip);

  // ---- cluster roles
  py::class_<Master>(m, "Master", py::module_local())
      .def(py::init<const ConfigParser&>(), py::keep_alive<1, 2>())
      .def_property_readonly("addr", &Master::addr)
      .def("init", &Master::init, py::call_guard<py::gil_scoped_release>())
      .def("terminate", &Master::terminate, py::call_guard<py::gil_scoped_release>())
      .def("run", &Master::run, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("server_num", &Master::server_num)
      .def_property_readonly("worker_num", &Master::worker_num);
  py::class_<Server>(m, "Server", py::module_local())
      .def(py::init<const ConfigParser&, int>(), py::keep_alive<1, 2>())
      .def("connect", &Server::connect, py::call_guard<py::gil_scoped_release>())
      .def("wait_terminate", &Server::wait_terminate, py::arg("timeout") = 1e9,
           py::call_guard<py::gil_scoped_release>())
      .def("table", &Server::table, py::return_value_policy::reference_internal)
      .def("backup", &Server::backup)
      .def_property_readonly("push_count", &Server::push_count)
      .def_property_readonly("client_id", &Server::client_id);
  py::class_<WorkerClient>(m, "WorkerClient", py::module_local())
      .def(py::init<const ConfigParser&>(), py::keep_alive<1, 2>())
      .def("connect", &WorkerClient::connect, py::call_guard<py::gil_scoped_release>())
      .def("pull", [](WorkerClient& w, u64arr k) {
        std::vector<float> out;
        int d;
        {
          py::gil_scoped_release rel;
          d = w.pull(k.data(), (size_t)k.size(), out);
        }
        py::array_t<float> a({(py::ssize_t)k.size(), (py::ssize_t)(d ? d : 1)});
        if (!out.empty()) std::memcpy(a.mutable_data(), out.data(), out.size() * 4);
        return a;
      })
      .def("push", [](WorkerClient& w, u64arr k, f32arr g) {
        const int d = k.size() ? (int)(g.size() / k.size()) : 1;
        py::gil_scoped_release rel;
        w.push(k.data(), (size_t)k.size(), g.data(), d);
      })
      .def("finish", &WorkerClient::finish, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("client_id", &WorkerClient::client_id)
      .def("server_ids", [](WorkerClient& w) { return w.route().server_ids; })
      .def("worker_ids", [](WorkerClient& w) { return w.route().worker_ids; })
      .def("hashfrag", [](WorkerClient& w) { return w.hashfrag(); });

  // ---- concurrency primitives (exposed for tests / apps)
  py::class_<ThreadPool>(m, "ThreadPool", py::module_local())
      .def(py::init<int>())
      .def("parallel_for", [](ThreadPool& p, int n, std::function<void(int)> f) {
        py::gil_scoped_release rel;
        p.parallel_for(n, [&f](int i) {
          py::gil_scoped_acquire g;
          f(i);
        });
      })
      .def("size", &ThreadPool::size)
      .def("stop", &ThreadPool::stop);
  // ---- data input (dataio.h)
  py::class_<SparseDataset>(m, "SparseDataset", py::module_local())
      .def(py::init<const std::string&, const std::string&, int, int, int>(), py::arg("path"),
           py::arg("format") = "libsvm", py::arg("nthreads") = 8, py::arg("shard") = 0,
           py::arg("nshards") = 1, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rows", &SparseDataset::rows)
      .def_property_readonly("nnz", &SparseDataset::nnz)
      .def_property_readonly("max_nnz", &SparseDataset::max_nnz)
      .def_property_readonly("has_values", &SparseDataset::has_values)
      .def("labels", [](const SparseDataset& d) {
        return py::array_t<float>(d.labels().size(), d.labels().data());
      })
      .def("keys", [](const SparseDataset& d) {
        return py::array_t<uint64_t>(d.keys().size(), d.keys().data());
      })
      .def("vals", [](const SparseDataset& d) {
        return py::array_t<float>(d.vals().size(), d.vals().data());
      })
      .def("offsets", [](const SparseDataset& d) {
        return py::array_t<uint64_t>(d.offsets().size(), d.offsets().data());
      })
      .def("fill", [](const SparseDataset& d, uint64_t cursor, int B, int F, uintptr_t keys,
                      uintptr_t vals, uintptr_t labels, int nthreads) {
             return d.fill(cursor, B, F, reinterpret_cast<uint64_t*>(keys),
                           reinterpret_cast<float*>(vals), reinterpret_cast<float*>(labels),
                           nthreads);
           }, py::arg("cursor"), py::arg("B"), py::arg("F"), py::arg("keys"), py::arg("vals"),
           py::arg("labels"), py::arg("nthreads") = 4, py::call_guard<py::gil_scoped_release>());

  py::class_<Corpus>(m, "Corpus", py::module_local())
      .def(py::init<const std::string&, int, int, int, int, double>(), py::arg("path"),
           py::arg("nthreads") = 8, py::arg("shard") = 0, py::arg("nshards") = 1,
           py::arg("min_count") = 1, py::arg("sample") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("size", &Corpus::size)
      .def_property_readonly("sentences", &Corpus::sentences)
      .def_property_readonly("vocab_size", &Corpus::vocab_size)
      .def("vocab", &Corpus::vocab)
      .def("tokens", [](const Corpus& c) {
        return py::array_t<uint64_t>(c.tokens().size(), c.tokens().data());
      })
      .def("sent_offsets", [](const Corpus& c) {
        return py::array_t<uint64_t>(c.sent_offsets().size(), c.sent_offsets().data());
      })
      .def("sent_of", [](const Corpus& c) {
        return py::array_t<uint32_t>(c.sent_of().size(), c.sent_of().data());
      })
      .def("noise_table", [](const Corpus& c) {
        return py::array_t<uint64_t>(c.noise_table().size(), c.noise_table().data());
      })
      .def_property_readonly("subsampled", &Corpus::subsampled)
      .def("keep_per_token", [](const Corpus& c) {
        auto k = c.keep_per_token();
        return py::array_t<float>(k.size(), k.data());
      })
      .def("fill_skipgram_window", [](const Corpus& c, uint64_t seed, uint64_t step, int B, int W,
                                      long long nneg, uintptr_t keys, uintptr_t meta) {
             if (W < 1 || W > kW2vMaxWindow) throw std::invalid_argument("window must be in [1, 15]");
             if (c.size() == 0) throw std::invalid_argument("empty corpus");
             c.fill_skipgram_window(seed, step, B, W, nneg, reinterpret_cast<uint64_t*>(keys),
                                    reinterpret_cast<int32_t*>(meta));
           }, py::arg("seed"), py::arg("step"), py::arg("B"), py::arg("W"), py::arg("nneg"),
           py::arg("keys"), py::arg("meta"), py::call_guard<py::gil_scoped_release>())
      .def("fill_skipgram", [](const Corpus& c, uint64_t seed, uint64_t step, int B, int C, int W,
                               long long nneg, uintptr_t keys, int nthreads) {
             c.fill_skipgram(seed, step, B, C, W, nneg, reinterpret_cast<uint64_t*>(keys),
                             nthreads);
           }, py::arg("seed"), py::arg("step"), py::arg("B"), py::arg("C"), py::arg("W"),
           py::arg("nneg"), py::arg("keys"), py::arg("nthreads") = 4,
           py::call_guard<py::gil_scoped_release>());

  m.def("channel_selftest", [](int producers, int items) {
    // MPMC stress: every produced item is consumed exactly once, close drains
    Channel<long> ch(64);
    std::atomic<long> sum{0};
    std::vector<std::thread> ps, cs;
    for (int p = 0; p < producers; ++p)
      ps.emplace_back([&, p] { for (int i = 0; i < items; ++i) ch.push((long)p * items + i); });
    for (int c = 0; c < 4; ++c)
      cs.emplace_back([&] { long v; while (ch.pop(v)) sum += v; });
    for (auto& t : ps) t.join();
    ch.close();
    for (auto& t : cs) t.join();
    return sum.load();
  }, py::call_guard<py::gil_scoped_release>());
}
