// SPDX-License-Identifier: Apache-2.0
// Local single-node (or simulated multi-node) cluster backend.
//
// Wires the object store (API server), pdo-kv, the gang scheduler, one
// agent per node (kubelet-lite) and the PaddleJob controller into a loop.
// Driven either by `tick()` (deterministic: tests, virtual clock) or by
// `start()` (daemon threads: pdo-manager --backend=local).
#pragma once

#include <atomic>
#include <memory>
#include <thread>
#include <vector>

#include "agent.h"
#include "controller.h"
#include "hostport.h"
#include "kvclient.h"
#include "kvstore.h"
#include "scheduler.h"
#include "store.h"

namespace pdo {

struct ClusterOptions {
  plan::Mode mode = plan::Mode::Fast;
  std::string init_image;   // "" = no coordinator (fast default); compat default busybox
  bool init_image_set = false;
  bool volcano = false;
  bool elastic_kv = true;   // in-process pdo-kv as the elastic store
  int workers = 1;
  bool virtual_clock = false;
  AgentOptions::Mode agent_mode = AgentOptions::Sim;
  std::vector<NodeInfo> nodes;     // default: one node "local" with 8 GPUs
  std::string sandbox_root = "/tmp/pdo-agent";
  double sim_ip_delay = 0.0, sim_start_delay = 0.0, sim_run_s = -1;
  double kubelet_config_retry_s = -1;  // <0: mode default (compat 1 s, fast event-driven)
  int port_start = 35000, port_end = 65000;
  std::string namespace_;
  std::string kv_endpoint = "127.0.0.1:2379";  // advertised to elastic pods (PADDLE_ELASTIC_SERVER)
  std::vector<std::string> zygote_cmd;          // per-node warm launcher (exec agents)
  bool start_gate = true;
  int ip_block_base = 1;                        // pods get 127.<base+node>.x.y                       // fast mode: native ps → worker → heter barrier
  // false: serve only the API server, gang scheduler, KV and kubelet-lite
  // agents — a single-node cluster for an external operator (e.g. pdo-manager
  // --backend=k8s pointed at this API), with no in-process PaddleJob controller
  bool controller = true;
};

class Cluster {
 public:
  explicit Cluster(ClusterOptions opt);
  ~Cluster();

  // one round of every component; returns true if anything progressed
  bool tick();
  // virtual clock
  double now() const;
  void advance(double dt);
  // drive until no progress (or virtual `max_s` elapsed); returns ticks run
  int settle(double max_s = 5.0);
  // tick for `s` seconds (virtual or real) regardless of quiescence
  int run_for(double s, double step = 0.01);
  void start();  // background loop (real clock)
  bool zygotes_ready() const;
  void stop();

  store::Store& store() { return *store_; }
  kv::KVStore& kv() { return *kv_; }
  Controller& controller() { return *ctrl_; }
  Scheduler& scheduler() { return *sched_; }
  Agent& agent(size_t i = 0) { return *agents_.at(i); }
  size_t num_agents() const { return agents_.size(); }
  HostPorts& ports() { return ports_; }
  const ClusterOptions& options() const { return opt_; }

  // kubectl-apply semantics for any object (create, or update spec/labels/annotations)
  json::Value apply(const std::string& kind, json::Value obj);
  bool exec(const std::string& ns, const std::string& pod, const std::string& container,
            const std::vector<std::string>& argv);
  Agent* agent_for(const std::string& ns, const std::string& pod);
  // every store event is also handed to this tap (HTTP watchers)
  void set_event_tap(std::function<void(const store::WatchEvent&)> tap) { tap_ = std::move(tap); }

 private:
  std::function<void(const store::WatchEvent&)> tap_;
  ClusterOptions opt_;
  std::atomic<double> vnow_{0};
  api::Clock clock_;
  std::unique_ptr<store::Store> store_;
  std::unique_ptr<kv::KVStore> kv_;
  std::unique_ptr<kv::LocalClient> kvc_;
  HostPorts ports_;
  std::unique_ptr<StoreApi> api_;
  std::unique_ptr<Scheduler> sched_;
  std::vector<std::unique_ptr<Agent>> agents_;
  std::unique_ptr<Controller> ctrl_;
  std::atomic<bool> running_{false};
  std::thread loop_;
  std::mutex tick_mu_;
};

}  // namespace pdo
