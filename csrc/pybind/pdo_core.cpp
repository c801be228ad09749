// SPDX-License-Identifier: Apache-2.0
// Python binding of the native control plane (paddle_operator_amd._pdo_core).
// Objects cross the boundary as plain Python dict/list/str/int/float/bool.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>

#include "apiserver.h"
#include "builders.h"
#include "cluster.h"
#include "http.h"
#include "kvclient.h"
#include "kvstore.h"
#include "metrics.h"
#include "planner.h"
#include "quantity.h"
#include "status.h"

namespace py = pybind11;
using pdo::json::Value;

static Value to_value(const py::handle& o) {
  if (o.is_none()) return Value();
  if (py::isinstance<py::bool_>(o)) return Value(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) return Value((int64_t)o.cast<long long>());
  if (py::isinstance<py::float_>(o)) return Value(o.cast<double>());
  if (py::isinstance<py::str>(o)) return Value(o.cast<std::string>());
  if (py::isinstance<py::bytes>(o)) return Value(o.cast<std::string>());
  if (py::isinstance<py::dict>(o)) {
    Value v = Value::object();
    for (auto item : o.cast<py::dict>()) v[py::str(item.first).cast<std::string>()] = to_value(item.second);
    return v;
  }
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    Value v = Value::array();
    for (auto item : o) v.push_back(to_value(item));
    return v;
  }
  throw py::type_error("unsupported type for JSON conversion");
}

static py::object to_py(const Value& v) {
  switch (v.type()) {
    case Value::Type::Null: return py::none();
    case Value::Type::Bool: return py::bool_(v.as_bool());
    case Value::Type::Int: return py::int_((long long)v.as_int());
    case Value::Type::Double: return py::float_(v.as_double());
    case Value::Type::String: return py::str(v.as_string());
    case Value::Type::Array: {
      py::list l;
      for (auto& x : v.arr()) l.append(to_py(x));
      return l;
    }
    case Value::Type::Object: {
      py::dict d;
      for (auto& m : v.obj()) d[py::str(m.first)] = to_py(m.second);
      return d;
    }
  }
  return py::none();
}

static pdo::api::PaddleJob job_of(const py::object& o) { return pdo::api::PaddleJob::from_json(to_value(o)); }

static pdo::build::Options build_opts(const py::dict& d) {
  pdo::build::Options o;
  if (d.contains("init_image")) o.init_image = d["init_image"].cast<std::string>();
  if (d.contains("volcano")) o.volcano = d["volcano"].cast<bool>();
  if (d.contains("etcd_endpoints")) o.etcd_endpoints = d["etcd_endpoints"].cast<std::vector<std::string>>();
  if (d.contains("gpu_resource_rewrite")) o.gpu_resource_rewrite = d["gpu_resource_rewrite"].cast<bool>();
  if (d.contains("launcher_env")) o.launcher_env = d["launcher_env"].cast<bool>();
  return o;
}

static pdo::plan::Options plan_opts(const py::dict& d) {
  std::string mode = d.contains("mode") ? d["mode"].cast<std::string>() : "fast";
  pdo::plan::Options o = mode == "compat" ? pdo::plan::Options::compat_defaults() : pdo::plan::Options::fast_defaults();
  pdo::build::Options b = build_opts(d);
  if (d.contains("init_image")) o.build.init_image = b.init_image;
  if (d.contains("etcd_endpoints")) o.build.etcd_endpoints = b.etcd_endpoints;
  if (d.contains("gpu_resource_rewrite")) o.build.gpu_resource_rewrite = b.gpu_resource_rewrite;
  if (d.contains("launcher_env")) o.build.launcher_env = b.launcher_env;
  if (d.contains("volcano")) o.volcano = d["volcano"].cast<bool>();
  if (d.contains("kv")) o.kv = d["kv"].cast<bool>();
  if (d.contains("compat_phase_lag")) o.sync.compat_phase_lag = d["compat_phase_lag"].cast<bool>();
  return o;
}

static py::dict action_dict(const pdo::plan::Action& a) {
  py::dict d;
  d["op"] = pdo::plan::op_name(a.op);
  d["name"] = a.name;
  d["role"] = a.role;
  d["detail"] = a.detail;
  d["obj"] = to_py(a.obj);
  d["targets"] = a.targets;
  return d;
}

static pdo::ClusterOptions cluster_opts(const py::kwargs& kw) {
  pdo::ClusterOptions o;
  for (auto item : kw) {
    const std::string k = py::str(item.first);
    const py::handle v = item.second;
    if (k == "mode") o.mode = v.cast<std::string>() == "compat" ? pdo::plan::Mode::Compat : pdo::plan::Mode::Fast;
    else if (k == "init_image") {
      o.init_image = v.cast<std::string>();
      o.init_image_set = true;
    } else if (k == "volcano") o.volcano = v.cast<bool>();
    else if (k == "elastic_kv") o.elastic_kv = v.cast<bool>();
    else if (k == "workers") o.workers = v.cast<int>();
    else if (k == "virtual_clock") o.virtual_clock = v.cast<bool>();
    else if (k == "agent") o.agent_mode = v.cast<std::string>() == "exec" ? pdo::AgentOptions::Exec : pdo::AgentOptions::Sim;
    else if (k == "sandbox_root") o.sandbox_root = v.cast<std::string>();
    else if (k == "sim_ip_delay") o.sim_ip_delay = v.cast<double>();
    else if (k == "sim_start_delay") o.sim_start_delay = v.cast<double>();
    else if (k == "sim_run_s") o.sim_run_s = v.cast<double>();
    else if (k == "kubelet_config_retry_s") o.kubelet_config_retry_s = v.cast<double>();
    else if (k == "port_range") {
      auto pr = v.cast<std::pair<int, int>>();
      o.port_start = pr.first;
      o.port_end = pr.second;
    } else if (k == "namespace") o.namespace_ = v.cast<std::string>();
    else if (k == "kv_endpoint") o.kv_endpoint = v.cast<std::string>();
    else if (k == "zygote_cmd") o.zygote_cmd = v.cast<std::vector<std::string>>();
    else if (k == "start_gate") o.start_gate = v.cast<bool>();
    else if (k == "ip_block_base") o.ip_block_base = v.cast<int>();
    else if (k == "nodes") {
      for (auto n : v.cast<py::list>()) {
        auto d = n.cast<py::dict>();
        pdo::NodeInfo ni;
        if (d.contains("name")) ni.name = d["name"].cast<std::string>();
        if (d.contains("ip")) ni.ip = d["ip"].cast<std::string>();
        if (d.contains("gpus")) ni.gpus = d["gpus"].cast<int>();
        if (d.contains("gpu_cpulists")) ni.gpu_cpulists = d["gpu_cpulists"].cast<std::vector<std::string>>();
        o.nodes.push_back(ni);
      }
    } else {
      throw py::key_error("unknown Cluster option " + k);
    }
  }
  return o;
}

// a Cluster plus its optional HTTP front end
struct PyCluster {
  std::unique_ptr<pdo::Cluster> c;
  std::unique_ptr<pdo::http::Server> srv;
  std::unique_ptr<pdo::WatchHub> hub;
};

struct PyKVServer {
  std::unique_ptr<pdo::kv::KVStore> store;
  std::unique_ptr<pdo::http::Server> srv;
  std::atomic<bool> run{false};
  std::thread expirer;
  ~PyKVServer() {
    run = false;
    if (expirer.joinable()) expirer.join();
    if (srv) srv->stop();
  }
};

PYBIND11_MODULE(_pdo_core, m) {
  m.doc() = "paddle_operator_amd native control plane (C++17)";
  py::register_exception<pdo::store::ApiError>(m, "ApiError");
  py::register_exception<pdo::json::ParseError>(m, "JSONParseError", PyExc_ValueError);

  // ---- builders / FSM / planner (pure)
  m.def("res_name", &pdo::build::res_name);
  m.def("extract_name_index", &pdo::build::extract_name_index);
  m.def("endpoints_to_hosts", &pdo::build::endpoints_to_hosts);
  m.def("construct_pod", [](py::object job, const std::string& role, int idx, py::dict opts) {
    return to_py(pdo::build::construct_pod(job_of(job), role, idx, build_opts(opts)));
  }, py::arg("job"), py::arg("role"), py::arg("idx"), py::arg("opts") = py::dict());
  m.def("construct_configmap", [](py::object job, py::list pods) {
    std::vector<Value> ps;
    for (auto p : pods) ps.push_back(to_value(p));
    return to_py(pdo::build::construct_configmap(job_of(job), ps));
  });
  m.def("construct_service_for_pod", [](py::object pod) {
    return to_py(pdo::build::construct_service_for_pod(to_value(pod)));
  });
  m.def("construct_podgroup", [](py::object job, bool rewrite) {
    return to_py(pdo::build::construct_podgroup(job_of(job), rewrite));
  }, py::arg("job"), py::arg("rewrite_gpu") = true);
  m.def("pg_min_resources", [](py::object job, bool rewrite) {
    return to_py(pdo::build::pg_min_resources(job_of(job), rewrite));
  }, py::arg("job"), py::arg("rewrite_gpu") = true);
  m.def("without_volcano", [](py::object job) { return pdo::build::without_volcano(job_of(job)); });
  m.def("validate", [](py::object job) { return pdo::api::validate(job_of(job)); });
  m.def("normalize", [](py::object job) { return to_py(job_of(job).to_json()); },
        "round-trip a PaddleJob through the typed schema (omitempty rules)");
  m.def("derive_phase", [](py::object job) { return pdo::fsm::derive_phase(job_of(job)); });
  m.def("derive_mode", [](py::object job) { return pdo::fsm::derive_mode(job_of(job).spec); });
  m.def("pod_really_running", [](py::object pod) { return pdo::fsm::pod_really_running(to_value(pod)); });
  m.def("coord_running", [](py::object pod) { return pdo::fsm::coord_running(to_value(pod)); });
  m.def("sync_status", [](py::object job, py::list pods, double now, bool compat) {
    std::vector<Value> ps;
    for (auto p : pods) ps.push_back(to_value(p));
    pdo::fsm::SyncOptions o;
    o.compat_phase_lag = compat;
    if (compat) {
      o.count_unknown = false;
      o.set_observed_generation = false;
    }
    return to_py(pdo::fsm::sync_status(job_of(job), ps, now, o).to_json());
  }, py::arg("job"), py::arg("pods"), py::arg("now"), py::arg("compat") = false);
  m.def("quantity_sum", [](std::vector<std::string> qs) {
    pdo::Quantity acc;
    bool first = true;
    for (auto& s : qs) {
      pdo::Quantity q;
      if (!pdo::Quantity::parse(s, &q)) throw py::value_error("bad quantity " + s);
      if (first) acc = q;
      else acc.add(q);
      first = false;
    }
    return acc.str();
  });

  py::class_<pdo::HostPorts>(m, "HostPorts")
      .def(py::init<int, int>(), py::arg("start") = 35000, py::arg("end") = 65000)
      .def("allocate", &pdo::HostPorts::allocate)
      .def("registered", &pdo::HostPorts::registered)
      .def("register_port", &pdo::HostPorts::register_port)
      .def("release", &pdo::HostPorts::release)
      .def("__len__", &pdo::HostPorts::size);

  m.def("plan", [](py::dict observed, py::dict options, pdo::HostPorts* ports, double now) {
    pdo::plan::Observed obs;
    obs.job = job_of(observed["job"]);
    if (observed.contains("pods"))
      for (auto p : observed["pods"].cast<py::list>()) obs.pods.push_back(to_value(p));
    if (observed.contains("services"))
      for (auto p : observed["services"].cast<py::list>()) obs.services.push_back(to_value(p));
    if (observed.contains("configmap_exists")) obs.configmap_exists = observed["configmap_exists"].cast<bool>();
    if (observed.contains("podgroup_exists")) obs.podgroup_exists = observed["podgroup_exists"].cast<bool>();
    if (observed.contains("podgroup_phase")) obs.podgroup_phase = observed["podgroup_phase"].cast<std::string>();
    if (observed.contains("kv_ok")) obs.kv_ok = observed["kv_ok"].cast<bool>();
    if (observed.contains("kv_count")) obs.kv_count = observed["kv_count"].cast<int>();
    if (observed.contains("kv_np")) obs.kv_np = observed["kv_np"].cast<std::string>();
    pdo::plan::Plan p = pdo::plan::reconcile(obs, plan_opts(options), ports, now);
    py::dict out;
    py::list acts;
    for (auto& a : p.actions) acts.append(action_dict(a));
    out["actions"] = acts;
    out["requeue"] = p.requeue;
    out["requeue_after"] = p.requeue_after;
    out["step"] = p.step;
    out["status"] = to_py(p.status.to_json());
    out["status_changed"] = p.status_changed;
    return out;
  }, py::arg("observed"), py::arg("options") = py::dict(), py::arg("ports") = nullptr, py::arg("now") = 0.0);

  // ---- KV store + etcd JSON gateway
  py::class_<pdo::kv::KVStore>(m, "KVStore")
      .def(py::init<>())
      .def("put", [](pdo::kv::KVStore& s, const std::string& k, const std::string& v, int64_t lease) {
        return s.put(k, v, lease);
      }, py::arg("key"), py::arg("value"), py::arg("lease") = 0)
      .def("get", [](pdo::kv::KVStore& s, const std::string& k) -> py::object {
        pdo::kv::KeyValue kv;
        if (!s.get(k, &kv)) return py::none();
        return py::str(kv.value);
      })
      .def("range", [](pdo::kv::KVStore& s, const std::string& k, const std::string& end) {
        py::list out;
        for (auto& kv : s.range(k, end)) out.append(py::make_tuple(kv.key, kv.value, kv.mod_revision, kv.version));
        return out;
      }, py::arg("key"), py::arg("range_end") = "")
      .def("prefix", [](pdo::kv::KVStore& s, const std::string& p) {
        py::dict out;
        for (auto& kv : s.range(p, pdo::kv::KVStore::prefix_end(p))) out[py::str(kv.key)] = py::str(kv.value);
        return out;
      })
      .def("delete", [](pdo::kv::KVStore& s, const std::string& k, const std::string& end) {
        return s.delete_range(k, end);
      }, py::arg("key"), py::arg("range_end") = "")
      .def("cas", [](pdo::kv::KVStore& s, const std::string& k, int64_t expect_version, const std::string& v) {
        pdo::kv::Compare c;
        c.key = k;
        c.target = pdo::kv::Compare::Version;
        c.num = expect_version;
        pdo::kv::Op op;
        op.type = pdo::kv::Op::Put;
        op.key = k;
        op.value = v;
        return s.txn({c}, {op}, {}, nullptr);
      })
      .def("lease_grant", &pdo::kv::KVStore::lease_grant, py::arg("ttl"), py::arg("id") = 0)
      .def("lease_revoke", &pdo::kv::KVStore::lease_revoke)
      .def("lease_keepalive", &pdo::kv::KVStore::lease_keepalive)
      .def("expire_leases", &pdo::kv::KVStore::expire_leases)
      .def("revision", &pdo::kv::KVStore::revision)
      .def_static("prefix_end", &pdo::kv::KVStore::prefix_end);

  py::class_<PyKVServer>(m, "KVServer")
      .def(py::init([](const std::string& addr) {
        auto s = new PyKVServer();
        s->store.reset(new pdo::kv::KVStore());
        s->srv.reset(new pdo::http::Server());
        pdo::kv::mount_gateway(*s->srv, *s->store);
        s->srv->route("GET", "/metrics", [](const pdo::http::Request&) {
          pdo::http::Response r;
          r.content_type = "text/plain; version=0.0.4";
          r.body = pdo::Metrics::global().expose();
          return r;
        });
        if (s->srv->listen(addr) < 0) {
          delete s;
          throw std::runtime_error("KVServer: cannot listen on " + addr);
        }
        s->srv->start();
        s->run = true;
        pdo::kv::KVStore* st = s->store.get();
        std::atomic<bool>* run = &s->run;
        s->expirer = std::thread([st, run] {
          while (*run) {
            st->expire_leases();
            usleep(100000);
          }
        });
        return s;
      }), py::arg("addr") = "127.0.0.1:0")
      .def_property_readonly("port", [](PyKVServer& s) { return s.srv->port(); })
      .def_property_readonly("store", [](PyKVServer& s) { return s.store.get(); }, py::return_value_policy::reference)
      .def("stop", [](PyKVServer& s) {
        s.run = false;
        if (s.expirer.joinable()) s.expirer.join();
        s.srv->stop();
      });

  // ---- local cluster backend
  py::class_<PyCluster>(m, "Cluster")
      .def(py::init([](py::kwargs kw) {
        auto c = new PyCluster();
        c->c.reset(new pdo::Cluster(cluster_opts(kw)));
        return c;
      }))
      .def("create", [](PyCluster& c, const std::string& kind, py::object obj) {
        return to_py(c.c->store().create(kind, to_value(obj)));
      })
      .def("apply", [](PyCluster& c, const std::string& kind, py::object obj) {
        return to_py(c.c->apply(kind, to_value(obj)));
      })
      .def("get", [](PyCluster& c, const std::string& kind, const std::string& ns, const std::string& name) -> py::object {
        Value v;
        if (!c.c->store().try_get(kind, ns, name, &v)) return py::none();
        return to_py(v);
      })
      .def("list", [](PyCluster& c, const std::string& kind, const std::string& ns, py::dict labels,
                      const std::string& owner) {
        std::map<std::string, std::string> l;
        for (auto item : labels) l[py::str(item.first)] = py::str(item.second);
        py::list out;
        for (auto& v : c.c->store().list(kind, ns, l, owner)) out.append(to_py(v));
        return out;
      }, py::arg("kind"), py::arg("ns") = "", py::arg("labels") = py::dict(), py::arg("owner") = "")
      .def("update", [](PyCluster& c, const std::string& kind, py::object obj) {
        return to_py(c.c->store().update(kind, to_value(obj)));
      })
      .def("update_status", [](PyCluster& c, const std::string& kind, py::object obj) {
        return to_py(c.c->store().update_status(kind, to_value(obj)));
      })
      .def("delete", [](PyCluster& c, const std::string& kind, const std::string& ns, const std::string& name) {
        Value cur;
        if (!c.c->store().try_get(kind, ns, name, &cur)) return false;
        c.c->store().remove(kind, ns, name, kind == "Pod" && cur.at_path("spec.nodeName").is_string());
        return true;
      })
      .def("tick", [](PyCluster& c) {
        py::gil_scoped_release g;
        return c.c->tick();
      })
      .def("settle", [](PyCluster& c, double max_s) {
        py::gil_scoped_release g;
        return c.c->settle(max_s);
      }, py::arg("max_s") = 5.0)
      .def("run_for", [](PyCluster& c, double s, double step) {
        py::gil_scoped_release g;
        return c.c->run_for(s, step);
      }, py::arg("seconds"), py::arg("step") = 0.01)
      .def("now", [](PyCluster& c) { return c.c->now(); })
      .def("advance", [](PyCluster& c, double dt) { c.c->advance(dt); })
      .def("exec", [](PyCluster& c, const std::string& ns, const std::string& pod, const std::string& container,
                      std::vector<std::string> argv) {
        py::gil_scoped_release g;
        return c.c->exec(ns, pod, container, argv);
      })
      .def("kill", [](PyCluster& c, const std::string& ns, const std::string& pod, int sig) {
        pdo::Agent* a = c.c->agent_for(ns, pod);
        return a && a->kill_pod(ns, pod, sig);
      }, py::arg("ns"), py::arg("pod"), py::arg("sig") = 9)
      .def("sim_exit", [](PyCluster& c, const std::string& ns, const std::string& pod, int code) {
        pdo::Agent* a = c.c->agent_for(ns, pod);
        return a && a->sim_exit(ns, pod, code);
      }, py::arg("ns"), py::arg("pod"), py::arg("code") = 0)
      .def("sandbox", [](PyCluster& c, const std::string& ns, const std::string& pod) {
        pdo::Agent* a = c.c->agent_for(ns, pod);
        return a ? a->sandbox_of(ns, pod) : std::string();
      })
      .def("kv_put", [](PyCluster& c, const std::string& k, const std::string& v) { return c.c->kv().put(k, v); })
      .def("kv_get", [](PyCluster& c, const std::string& k) -> py::object {
        pdo::kv::KeyValue kv;
        if (!c.c->kv().get(k, &kv)) return py::none();
        return py::str(kv.value);
      })
      .def("kv_delete", [](PyCluster& c, const std::string& k) { return c.c->kv().delete_range(k); })
      .def("host_ports", [](PyCluster& c) { return c.c->ports().size(); })
      .def("free_gpus", [](PyCluster& c) { return c.c->scheduler().free_gpus(); })
      .def("queue_len", [](PyCluster& c) { return c.c->controller().queue().len(); })
      .def("reconcile", [](PyCluster& c, const std::string& ns, const std::string& name) {
        decltype(c.c->controller().reconcile(ns, name)) r;
        {
          py::gil_scoped_release g;
          r = c.c->controller().reconcile(ns, name);
        }
        return py::make_tuple(r.step, r.requeue, r.requeue_after, r.error, r.actions);
      })
      .def("serve", [](PyCluster& c, const std::string& addr) {
        c.hub.reset(new pdo::WatchHub());
        c.srv.reset(new pdo::http::Server());
        pdo::mount_apiserver(*c.srv, c.c->store(), *c.hub, c.c.get());
        pdo::kv::mount_gateway(*c.srv, c.c->kv());
        c.srv->route("GET", "/metrics", [](const pdo::http::Request&) {
          pdo::http::Response r;
          r.content_type = "text/plain; version=0.0.4";
          r.body = pdo::Metrics::global().expose();
          return r;
        });
        for (const char* p : {"/healthz", "/readyz"})
          c.srv->route("GET", p, [](const pdo::http::Request&) {
            pdo::http::Response r;
            r.content_type = "text/plain";
            r.body = "ok";
            return r;
          });
        pdo::WatchHub* hub = c.hub.get();
        c.c->set_event_tap([hub](const pdo::store::WatchEvent& e) { hub->publish(e); });
        int port = c.srv->listen(addr);
        if (port < 0) throw std::runtime_error("cannot listen on " + addr);
        c.srv->start();
        return port;
      }, py::arg("addr") = "127.0.0.1:0")
      .def("start", [](PyCluster& c) { c.c->start(); })
      .def("zygotes_ready", [](PyCluster& c) { return c.c->zygotes_ready(); })
      .def("stop", [](PyCluster& c) {
        py::gil_scoped_release g;
        c.c->stop();
        if (c.srv) c.srv->stop();
      });

  m.def("metrics", [] { return pdo::Metrics::global().expose(); });
  m.def("metrics_reset", [] { pdo::Metrics::global().reset(); });
  m.def("metric", [](const std::string& name, py::dict labels) {
    pdo::Labels l;
    for (auto item : labels) l[py::str(item.first)] = py::str(item.second);
    return pdo::Metrics::global().get(name, l);
  }, py::arg("name"), py::arg("labels") = py::dict());
  m.def("json_roundtrip", [](const std::string& s, int indent) { return Value::parse(s).dump(indent); },
        py::arg("text"), py::arg("indent") = -1);
}
