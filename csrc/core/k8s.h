// SPDX-License-Identifier: Apache-2.0
// Kubernetes REST backend: the same controller against a real apiserver.
//
// * Config: --master URL, --kubeconfig (YAML or JSON; token / client cert /
//   CA), or the in-cluster service account (KUBERNETES_SERVICE_HOST/PORT +
//   /var/run/secrets/kubernetes.io/serviceaccount).
// * Informer: LIST + WATCH per kind (PaddleJob, Pod, Service, ConfigMap
//   [, PodGroup]) mirrored into a local store::Store that the controller
//   reads (controller-runtime's cache), re-listing on watch expiry (410).
// * RestApi: writes (POST/PUT/PUT …/status/DELETE with Background
//   propagation) — the ObjectApi the controller's executor uses.
// * Leader election on a coordination.k8s.io/v1 Lease
//   (--leader-elect, id b2a304f2.paddlepaddle.org; main.go:93-94).
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "controller.h"
#include "http.h"
#include "store.h"

namespace pdo {
namespace k8s {

struct Config {
  std::string server;  // https://host:6443
  std::string token;
  std::string ca_file, cert_file, key_file;
  std::string ca_pem, cert_pem, key_pem;  // kubeconfig *-data: in memory only, never written to disk
  bool insecure = false;
  std::string ns = "default";  // namespace of the in-cluster pod (leases)
  static bool load(const std::string& kubeconfig, const std::string& master, Config* out, std::string* err);
  http::ClientOptions client(double timeout_s = 30) const;
};

class RestApi : public ObjectApi {
 public:
  explicit RestApi(Config c) : c_(std::move(c)) {}
  json::Value create(const std::string& kind, json::Value obj) override;
  json::Value update(const std::string& kind, json::Value obj) override;
  json::Value update_status(const std::string& kind, json::Value obj) override;
  void remove(const std::string& kind, const std::string& ns, const std::string& name, bool graceful) override;
  json::Value get(const std::string& kind, const std::string& ns, const std::string& name);
  json::Value list(const std::string& kind, const std::string& ns, std::string* rv);
  const Config& config() const { return c_; }

 private:
  json::Value call(const std::string& method, const std::string& path, const std::string& body);
  Config c_;
};

class Informer {
 public:
  Informer(RestApi* api, store::Store* cache, std::string kind, std::string ns)
      : api_(api), cache_(cache), kind_(std::move(kind)), ns_(std::move(ns)) {}
  ~Informer() { stop(); }
  void start();
  void stop();
  bool synced() const { return synced_; }
  int lists() const { return lists_; }      // LISTs issued (initial + relists)
  int watches() const { return watches_; }  // WATCH requests issued
  int watch_timeout_s = 300;

 private:
  void run();
  RestApi* api_;
  store::Store* cache_;
  std::string kind_, ns_;
  std::atomic<bool> running_{false}, synced_{false};
  std::atomic<int> lists_{0}, watches_{0};
  std::thread th_;
};

// one line of a watch stream (a watch.Event JSON) applied to the mirrored cache.
// *rv follows every event's metadata.resourceVersion, BOOKMARKs included.
// Returns false on an ERROR event (the stream is over), with *gone = 410
// Expired / Gone (the resourceVersion was compacted: relist).
bool apply_watch_event(const std::string& line, store::Store* cache, const std::string& kind, std::string* rv,
                       bool* gone);

class LeaderElector {
 public:
  LeaderElector(RestApi* api, std::string ns, std::string name, std::string identity)
      : api_(api), ns_(std::move(ns)), name_(std::move(name)), id_(std::move(identity)) {}
  // one acquire/renew attempt; true while we hold the lease
  bool try_acquire_or_renew(double now);
  double lease_duration = 15, renew_deadline = 10, retry_period = 2;

 private:
  RestApi* api_;
  std::string ns_, name_, id_;
  double last_renew_ = 0;
};

int run_manager(const std::string& kubeconfig, const std::string& master, const std::string& ns,
                const std::string& mode, bool volcano, const std::string& init_image, const std::string& etcd,
                int port_start, int port_end, bool leader_elect, const std::string& leader_id, int workers,
                std::atomic<bool>* stop, std::atomic<bool>* ready);

}  // namespace k8s
}  // namespace pdo
