// SPDX-License-Identifier: Apache-2.0
// PaddleJob controller: watches → workqueue → planner → executor.
//
// Counterpart of the reference's PaddleJobReconciler + SetupWithManager
// (controllers/paddlejob_controller.go:64-76,101-333,520-571): For(PaddleJob)
// .Owns(Pod, Service, ConfigMap[, PodGroup]) through the controller-owner
// index, events Created/Deleted/Create/Delete/Scaled, 1 s requeues on
// conflicts, rate-limited retries on errors.  Reads come from a cache
// (`store::Store`, fed either by the local backend directly or by the
// Kubernetes informer in k8s.cpp); writes go through an ObjectApi.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "hostport.h"
#include "objectapi.h"
#include "kvclient.h"
#include "planner.h"
#include "store.h"
#include "workqueue.h"

namespace pdo {

// kubectl exec <pod> -c <container> -- argv (coordinator release)
using ExecFn = std::function<bool(const std::string& ns, const std::string& pod, const std::string& container,
                                  const std::vector<std::string>& argv)>;

struct ControllerOptions {
  plan::Options plan = plan::Options::fast_defaults();
  std::string watch_namespace;  // --namespace ("" = all)
  int workers = 1;              // MaxConcurrentReconciles
  bool graceful_pod_delete = true;
  bool record_events = true;
};

struct ReconcileResult {
  bool requeue = false;
  double requeue_after = 0;
  bool error = false;
  std::string step;
  std::string message;
  int actions = 0;
};

class Controller {
 public:
  Controller(store::Store* cache, ObjectApi* api, kv::Client* kv, HostPorts* ports, ExecFn exec,
             ControllerOptions opt, api::Clock clock = api::wall_clock);
  ~Controller();

  // informer callback: map a watch event to PaddleJob keys
  void on_event(const store::WatchEvent& ev);
  // process one queued key (blocking up to timeout_s); false if none
  bool process_one(double timeout_s = 0);
  ReconcileResult reconcile(const std::string& ns, const std::string& name);
  void start();  // worker threads
  void stop();
  WorkQueue& queue() { return q_; }
  const ControllerOptions& options() const { return opt_; }
  void record_event(const json::Value& obj, const std::string& kind, const std::string& type,
                    const std::string& reason, const std::string& msg);

 private:
  void apply(const api::PaddleJob& job, json::Value raw, const plan::Plan& p, ReconcileResult* r);

  store::Store* cache_;
  ObjectApi* api_;
  kv::Client* kv_;
  HostPorts* ports_;
  ExecFn exec_;
  ControllerOptions opt_;
  api::Clock clock_;
  WorkQueue q_;
  std::vector<std::thread> workers_;
  std::atomic<bool> running_{false};
  std::map<std::string, std::string> last_phase_;  // for transition metrics
  std::map<std::string, double> first_seen_;
  std::mutex meta_mu_;
};

}  // namespace pdo
