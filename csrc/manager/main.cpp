// SPDX-License-Identifier: Apache-2.0
// pdo-manager: the PaddleJob operator process (reference: main.go).
//
// Flag parity with the reference (main.go:61-83):
//   --etcd-server --metrics-bind-address --namespace --health-probe-bind-address
//   --port-range --leader-elect --scheduling --initImage  (+ --zap-* flags)
// pdo additions:
//   --backend=local|k8s      local: built-in API server + kubelet-lite on this
//                            node (one rank per MI355X); k8s: a real cluster
//   --mode=fast|compat       launch path (compat = reference sequencing)
//   --api-bind-address       local backend REST API (k8s-compatible paths)
//   --agent=exec|sim --gpus N --sandbox-root DIR --workers N
//   --kubeconfig / --master  (k8s backend)
//   --apply FILE.json        create/update objects at start (local backend)
//   --controller=false       local backend as a bare single-node cluster (API
//                            server, scheduler, kubelet-lite, KV) for an external
//                            operator such as a second pdo-manager --backend=k8s
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <dirent.h>

#include <algorithm>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "apiserver.h"
#include "cluster.h"
#include "http.h"
#include "k8s.h"
#include "kvclient.h"
#include "log.h"
#include "metrics.h"

static std::atomic<bool> g_stop{false};
static void on_sig(int) { g_stop = true; }

struct Flags {
  std::string etcd_server;
  std::string metrics_addr = ":8080";
  std::string ns;
  std::string probe_addr = ":8081";
  std::string port_range = "35000,65000";
  bool leader_elect = false;
  std::string leader_id = "b2a304f2.paddlepaddle.org";
  std::string scheduling;
  std::string init_image = "docker.io/library/busybox:1";
  bool init_image_given = false;
  // pdo
  std::string backend = "local";
  std::string mode = "fast";
  std::string api_addr = "127.0.0.1:8082";
  std::string kv_addr;  // serve the in-process pdo-kv gateway (local backend)
  std::string agent = "exec";
  int gpus = -1;
  std::string sandbox_root = "/tmp/pdo-agent";
  int workers = 1;
  std::string kubeconfig, master;
  std::vector<std::string> apply;
  bool controller = true;  // --controller=false: local backend without its PaddleJob controller
};

static int detect_gpus() {
  // count AMD render nodes via KFD topology (no HIP init in the manager)
  int n = 0;
  DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
  if (!d) return 0;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::ifstream f(std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name + "/properties");
    std::string k;
    long long v;
    while (f >> k >> v)
      if (k == "simd_count" && v > 0) {
        ++n;
        break;
      }
  }
  closedir(d);
  // a restricted manager (container / scheduler slice) only owns what it sees
  for (const char* var : {"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"}) {
    const char* v = getenv(var);
    if (!v || !*v) continue;
    int cnt = 1;
    for (const char* q = v; *q; ++q) cnt += *q == ',';
    n = std::min(n, cnt);
  }
  return n;
}

// NUMA-local CPU list of every GPU, in KFD node order (= HIP device order),
// from sysfs: KFD node properties (domain, location_id = PCI bus/dev/fn) →
// /sys/bus/pci/devices/<bdf>/local_cpulist.  The kubelet-lite agent pins each
// rank process to the list of its GPU (agent.cpp start_proc).  Mapped through
// HIP_VISIBLE_DEVICES when the manager itself is restricted.
static std::vector<std::string> detect_gpu_cpulists() {
  std::vector<std::pair<long, std::string>> nodes;  // (kfd node id, cpulist)
  DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
  if (!d) return {};
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::ifstream f(std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name + "/properties");
    std::string k;
    long long v, simd = 0, loc = 0, dom = 0;
    while (f >> k >> v) {
      if (k == "simd_count") simd = v;
      else if (k == "location_id") loc = v;
      else if (k == "domain") dom = v;
    }
    if (simd <= 0) continue;
    char bdf[32];
    snprintf(bdf, sizeof bdf, "%04llx:%02llx:%02llx.%llx", dom, (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 0x7);
    std::ifstream c(std::string("/sys/bus/pci/devices/") + bdf + "/local_cpulist");
    std::string list;
    std::getline(c, list);
    nodes.emplace_back(strtol(e->d_name, nullptr, 10), list);
  }
  closedir(d);
  std::sort(nodes.begin(), nodes.end());
  std::vector<std::string> all;
  for (auto& n : nodes) all.push_back(n.second);
  const char* pv = getenv("HIP_VISIBLE_DEVICES");
  if (!pv || !*pv) pv = getenv("CUDA_VISIBLE_DEVICES");
  if (!pv || !*pv) return all;
  std::vector<std::string> out;
  std::string cur;
  for (const char* q = pv;; ++q) {
    if (*q == ',' || *q == 0) {
      const long i = cur.empty() ? -1 : strtol(cur.c_str(), nullptr, 10);
      out.push_back(i >= 0 && i < (long)all.size() ? all[i] : "");
      cur.clear();
      if (!*q) break;
    } else {
      cur += *q;
    }
  }
  return out;
}

static void usage() {
  printf(
      "pdo-manager — PaddleJob operator for MI355X clusters\n"
      "  --etcd-server URLS            elastic np store (default: in-process pdo-kv on local backend)\n"
      "  --metrics-bind-address ADDR   (:8080)\n  --health-probe-bind-address ADDR (:8081)\n"
      "  --namespace NS                watch only NS\n  --port-range A,B            host-network ports (35000,65000)\n"
      "  --leader-elect                Lease-based leader election\n  --scheduling volcano       gang scheduling\n"
      "  --initImage IMAGE             coordinator init image ('' disables)\n"
      "  --backend local|k8s  --mode fast|compat  --api-bind-address ADDR  --agent exec|sim\n"
      "  --gpus N  --sandbox-root DIR  --workers N  --kubeconfig F  --master URL  --apply FILE\n"
      "  --controller=false            local backend without its PaddleJob controller\n"
      "  --zap-log-level L  --zap-encoder json|console  --zap-devel\n");
}

int main(int argc, char** argv) {
  Flags f;
  pdo::log::Config lc;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    std::string flag = a, val;
    bool has_eq = false;
    size_t eq = a.find('=');
    if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
      flag = a.substr(0, eq);
      val = a.substr(eq + 1);
      has_eq = true;
    }
    if (flag.rfind("--", 0) != 0 && flag.rfind("-", 0) == 0) flag = "-" + flag;  // -flag → --flag (Go style)
    auto next = [&]() -> std::string {
      if (has_eq) return val;
      if (i + 1 < argc) return argv[++i];
      fprintf(stderr, "missing value for %s\n", flag.c_str());
      exit(2);
    };
    auto boolean = [&]() -> bool { return has_eq ? (val == "true" || val == "1") : true; };
    if (flag == "--etcd-server") f.etcd_server = next();
    else if (flag == "--metrics-bind-address") f.metrics_addr = next();
    else if (flag == "--namespace") f.ns = next();
    else if (flag == "--health-probe-bind-address") f.probe_addr = next();
    else if (flag == "--port-range") f.port_range = next();
    else if (flag == "--leader-elect") f.leader_elect = boolean();
    else if (flag == "--leader-election-id") f.leader_id = next();
    else if (flag == "--scheduling") f.scheduling = next();
    else if (flag == "--initImage" || flag == "--init-image") {
      f.init_image = next();
      f.init_image_given = true;
    } else if (flag == "--backend") f.backend = next();
    else if (flag == "--mode") f.mode = next();
    else if (flag == "--api-bind-address") f.api_addr = next();
    else if (flag == "--kv-bind-address") f.kv_addr = next();
    else if (flag == "--agent") f.agent = next();
    else if (flag == "--gpus") f.gpus = atoi(next().c_str());
    else if (flag == "--sandbox-root") f.sandbox_root = next();
    else if (flag == "--workers") f.workers = atoi(next().c_str());
    else if (flag == "--kubeconfig") f.kubeconfig = next();
    else if (flag == "--master") f.master = next();
    else if (flag == "--apply") f.apply.push_back(next());
    else if (flag == "--controller") f.controller = boolean();
    else if (flag == "--zap-log-level") {
      if (!pdo::log::parse_level(next(), &lc.level)) return 2;
    } else if (flag == "--zap-encoder") lc.json = next() == "json";
    else if (flag == "--zap-devel") lc.devel = boolean();
    else if (flag == "--zap-stacktrace-level" || flag == "--zap-time-encoding") next();
    else if (flag == "-h" || flag == "--help") {
      usage();
      return 0;
    } else {
      fprintf(stderr, "unknown flag %s\n", a.c_str());
      usage();
      return 2;
    }
  }
  pdo::log::configure(lc);
  const char* L = "setup";
  int ps = 0, pe = 0;
  if (!pdo::HostPorts::parse_range(f.port_range, &ps, &pe)) {
    pdo::log::error(L, "port should have int type", {{"port-range", f.port_range}});
    return 1;
  }
  signal(SIGTERM, on_sig);
  signal(SIGINT, on_sig);
  signal(SIGPIPE, SIG_IGN);

  // health / readiness probes + metrics (main.go:90,158-165)
  pdo::http::Server probes, metrics;
  std::atomic<bool> ready{false};
  probes.route("GET", "/healthz", [](const pdo::http::Request&) {
    pdo::http::Response r;
    r.content_type = "text/plain";
    r.body = "ok";
    return r;
  });
  probes.route("GET", "/readyz", [&ready](const pdo::http::Request&) {
    pdo::http::Response r;
    r.content_type = "text/plain";
    r.status = ready ? 200 : 503;
    r.body = ready ? "ok" : "not ready";
    return r;
  });
  metrics.route("GET", "/metrics", [](const pdo::http::Request&) {
    pdo::http::Response r;
    r.content_type = "text/plain; version=0.0.4";
    r.body = pdo::Metrics::global().expose();
    return r;
  });
  if (f.probe_addr != "0" && probes.listen(f.probe_addr) < 0) {
    pdo::log::error(L, "unable to bind health probe address", {{"addr", f.probe_addr}});
    return 1;
  }
  if (f.metrics_addr != "0" && metrics.listen(f.metrics_addr) < 0) {
    pdo::log::error(L, "unable to bind metrics address", {{"addr", f.metrics_addr}});
    return 1;
  }
  probes.start();
  metrics.start();

  if (f.backend == "k8s") {
    int rc = pdo::k8s::run_manager(f.kubeconfig, f.master, f.ns, f.mode, f.scheduling == "volcano",
                                   f.init_image_given ? f.init_image : (f.mode == "compat" ? f.init_image : ""),
                                   f.etcd_server, ps, pe, f.leader_elect, f.leader_id, f.workers, &g_stop, &ready);
    probes.stop();
    metrics.stop();
    return rc;
  }
  if (f.backend != "local") {
    pdo::log::error(L, "unknown backend", {{"backend", f.backend}});
    return 2;
  }

  pdo::ClusterOptions co;
  co.mode = f.mode == "compat" ? pdo::plan::Mode::Compat : pdo::plan::Mode::Fast;
  if (f.init_image_given) {
    co.init_image = f.init_image;
    co.init_image_set = true;
  }
  co.volcano = f.scheduling == "volcano";
  co.workers = f.workers;
  co.agent_mode = f.agent == "sim" ? pdo::AgentOptions::Sim : pdo::AgentOptions::Exec;
  co.sandbox_root = f.sandbox_root;
  co.port_start = ps;
  co.port_end = pe;
  co.namespace_ = f.ns;
  co.controller = f.controller;
  pdo::NodeInfo node;
  node.name = "local";
  node.gpus = f.gpus >= 0 ? f.gpus : detect_gpus();
  node.gpu_cpulists = detect_gpu_cpulists();
  if ((int)node.gpu_cpulists.size() > node.gpus) node.gpu_cpulists.resize(node.gpus);
  co.nodes.push_back(node);
  pdo::Cluster cluster(co);
  pdo::WatchHub hub;
  pdo::http::Server api;
  pdo::mount_apiserver(api, cluster.store(), hub, &cluster);
  pdo::kv::mount_gateway(api, cluster.kv());
  cluster.set_event_tap([&hub](const pdo::store::WatchEvent& e) { hub.publish(e); });
  if (api.listen(f.api_addr) < 0) {
    pdo::log::error(L, "unable to bind API address", {{"addr", f.api_addr}});
    return 1;
  }
  api.start();
  std::unique_ptr<pdo::http::Server> kvsrv;
  if (!f.kv_addr.empty()) {
    kvsrv.reset(new pdo::http::Server());
    pdo::kv::mount_gateway(*kvsrv, cluster.kv());
    if (kvsrv->listen(f.kv_addr) < 0) {
      pdo::log::error(L, "unable to bind kv address", {{"addr", f.kv_addr}});
      return 1;
    }
    kvsrv->start();
  }
  for (auto& file : f.apply) {
    std::ifstream in(file);
    std::string text((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    try {
      pdo::json::Value v = pdo::json::Value::parse(text);
      std::vector<pdo::json::Value> objs;
      if (v.get("kind").as_string() == "List") {
        for (auto& o : v.get("items").arr()) objs.push_back(o);
      } else {
        objs.push_back(v);
      }
      for (auto& o : objs) cluster.apply(o.get("kind").str(), o);
    } catch (const std::exception& e) {
      pdo::log::error(L, "apply failed", {{"file", file}, {"error", e.what()}});
      return 1;
    }
  }
  cluster.start();
  ready = true;
  pdo::log::info(L, "starting manager", {{"backend", "local"}, {"mode", f.mode},
                                          {"api", "http://" + f.api_addr}, {"gpus", std::to_string(node.gpus)}});
  while (!g_stop) usleep(100000);
  pdo::log::info(L, "shutting down");
  cluster.stop();
  api.stop();
  if (kvsrv) kvsrv->stop();
  probes.stop();
  metrics.stop();
  return 0;
}
