// SPDX-License-Identifier: Apache-2.0
#include "cluster.h"

#include <unistd.h>

#include <chrono>
#include <cmath>

#include "log.h"

namespace pdo {

using json::Value;

Cluster::Cluster(ClusterOptions opt) : opt_(std::move(opt)) {
  if (opt_.virtual_clock) {
    vnow_ = 1.7e9;
    clock_ = [this] { return vnow_.load(); };
  } else {
    clock_ = api::wall_clock;
  }
  if (opt_.nodes.empty()) {
    NodeInfo n;
    n.name = "local";
    n.gpus = 8;
    opt_.nodes.push_back(n);
  }
  store_.reset(new store::Store(clock_));
  kv_.reset(new kv::KVStore(clock_));
  kvc_.reset(new kv::LocalClient(kv_.get(), opt_.kv_endpoint));
  ports_.reset(opt_.port_start, opt_.port_end);
  api_.reset(new StoreApi(store_.get()));
  sched_.reset(new Scheduler(store_.get(), opt_.nodes));
  const bool compat = opt_.mode == plan::Mode::Compat;
  int block = opt_.ip_block_base;
  for (auto& n : opt_.nodes) {
    if (n.remote) continue;
    AgentOptions ao;
    ao.mode = opt_.agent_mode;
    ao.node = n;
    ao.sandbox_root = opt_.sandbox_root + "/" + n.name;
    ao.ip_block = block++;
    ao.sim_ip_delay = opt_.sim_ip_delay;
    ao.sim_start_delay = opt_.sim_start_delay;
    ao.sim_run_s = opt_.sim_run_s;
    ao.zygote_cmd = opt_.zygote_cmd;
    ao.config_retry_s = opt_.kubelet_config_retry_s >= 0 ? opt_.kubelet_config_retry_s : (compat ? 1.0 : 0.0);
    agents_.emplace_back(new Agent(store_.get(), ao, clock_));
  }
  ControllerOptions co;
  co.plan = compat ? plan::Options::compat_defaults() : plan::Options::fast_defaults();
  if (opt_.init_image_set) co.plan.build.init_image = opt_.init_image;
  // the local agent honours the native start gate; fast mode uses it instead of exec
  co.plan.build.start_gate = !compat && opt_.start_gate;
  co.plan.volcano = opt_.volcano;
  co.plan.kv = opt_.elastic_kv;
  if (opt_.elastic_kv) co.plan.build.etcd_endpoints = kvc_->endpoints();
  co.workers = opt_.workers;
  co.watch_namespace = opt_.namespace_;
  ExecFn ex = [this](const std::string& ns, const std::string& pod, const std::string& c,
                     const std::vector<std::string>& argv) { return exec(ns, pod, c, argv); };
  ctrl_.reset(new Controller(store_.get(), api_.get(), opt_.elastic_kv ? kvc_.get() : nullptr, &ports_, ex, co,
                             clock_));
}

Cluster::~Cluster() {
  stop();
  for (auto& a : agents_) a->shutdown();
}

double Cluster::now() const { return clock_(); }

bool Cluster::zygotes_ready() const {
  for (auto& a : agents_)
    if (!a->zygote_socket().empty() && !a->zygote_ready()) return false;
  return true;
}

void Cluster::advance(double dt) {
  if (!opt_.virtual_clock) return;
  double cur = vnow_.load();
  vnow_.store(cur + dt);
}

Agent* Cluster::agent_for(const std::string& ns, const std::string& pod) {
  Value p;
  if (!store_->try_get("Pod", ns, pod, &p)) return nullptr;
  const std::string node = p.at_path("spec.nodeName").str();
  for (auto& a : agents_)
    if (a->options().node.name == node) return a.get();
  return nullptr;
}

bool Cluster::exec(const std::string& ns, const std::string& pod, const std::string& container,
                   const std::vector<std::string>& argv) {
  Agent* a = agent_for(ns, pod);
  return a && a->exec(ns, pod, container, argv);
}

bool Cluster::tick() {
  std::lock_guard<std::mutex> g(tick_mu_);
  bool progress = false;
  // informers: deliver watch events
  auto evs = store_->drain();
  if (!evs.empty()) progress = true;
  for (auto& e : evs) {
    if (opt_.controller) ctrl_->on_event(e);
    if (tap_) tap_(e);
  }
  // reconcile every ready key once (workers run in start() mode instead)
  if (!running_ && opt_.controller) {
    ctrl_->queue().promote_due();
    int guard = 0;
    while (guard++ < 256 && ctrl_->process_one(0)) progress = true;
  }
  if (sched_->sync() > 0) progress = true;
  for (auto& a : agents_)
    if (a->sync() > 0) progress = true;
  kv_->expire_leases();
  if (store_->has_events()) progress = true;
  return progress;
}

int Cluster::settle(double max_s) {
  // run until quiescent: no progress, no delayed requeue pending
  const double t_end = now() + max_s;
  int n = 0, idle = 0;
  while (now() < t_end) {
    ++n;
    if (tick()) {
      idle = 0;
      continue;
    }
    ++idle;
    const double nr = ctrl_->queue().next_ready_in();
    const bool timers = !std::isinf(nr);
    if (!timers && idle >= 3) break;
    const double step = timers ? std::min(std::max(nr, 0.001), 0.05) : 0.005;
    if (opt_.virtual_clock) advance(step);
    else usleep((useconds_t)(step * 1e6));
  }
  return n;
}

int Cluster::run_for(double s, double step) {
  const double t_end = now() + s;
  int n = 0;
  while (now() < t_end) {
    ++n;
    tick();
    if (opt_.virtual_clock) advance(step);
    else usleep((useconds_t)(step * 1e6));
  }
  tick();
  return n;
}

void Cluster::start() {
  if (running_.exchange(true)) return;
  if (opt_.controller) ctrl_->start();
  loop_ = std::thread([this] {
    while (running_) {
      bool p = tick();
      if (!p) store_->wait_events(0.02);
    }
  });
}

void Cluster::stop() {
  if (!running_.exchange(false)) return;
  if (loop_.joinable()) loop_.join();
  if (opt_.controller) ctrl_->stop();
}

Value Cluster::apply(const std::string& kind, Value obj) {
  const std::string ns = obj.at_path("metadata.namespace").str("default");
  obj["metadata"]["namespace"] = ns;
  const std::string name = obj.at_path("metadata.name").str();
  Value cur;
  if (!store_->try_get(kind, ns, name, &cur)) return store_->create(kind, obj);
  Value next = cur;
  next["spec"] = obj.get("spec");
  if (obj.has("data")) next["data"] = obj.get("data");
  for (const char* f : {"labels", "annotations"})
    if (obj.at_path(std::string("metadata.") + f).is_object()) next["metadata"][f] = obj.at_path(std::string("metadata.") + f);
  return store_->update(kind, next);
}

}  // namespace pdo
