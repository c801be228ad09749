// SPDX-License-Identifier: Apache-2.0
// In-memory Kubernetes-style object store: the API server of the `local`
// cluster backend (envtest's kube-apiserver + etcd, plus what envtest lacks).
//
// Semantics reproduced from the apiserver as the reference controller relies
// on them (SURVEY §3.7 boundaries, §7.4 risk 1):
//  * create → AlreadyExists; uid, resourceVersion (global revision),
//    creationTimestamp, generation = 1
//  * update → Conflict on a stale resourceVersion; generation bumps when spec
//    changes; the status subresource is written only by update_status, and
//    update_status never touches metadata/spec
//  * delete → with finalizers (or `graceful` for pods bound to a kubelet) only
//    sets deletionTimestamp; final removal garbage-collects dependents whose
//    ownerReferences name the removed uid (background propagation)
//  * every mutation produces an ADDED / MODIFIED / DELETED watch event that is
//    queued and delivered by `drain()` on the consumer's thread (informer-like)
//  * field index on the controller owner name (`.metadata.controller`,
//    paddlejob_controller.go:57-59,520-553)
#pragma once

#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "api.h"
#include "json.h"

namespace pdo {
namespace store {

using json::Value;

class ApiError : public std::runtime_error {
 public:
  enum Code { NotFound = 404, AlreadyExists = 409, Conflict = 4090, Invalid = 422 };
  ApiError(Code c, const std::string& msg) : std::runtime_error(msg), code(c) {}
  Code code;
};

enum class EventType { Added, Modified, Deleted };
const char* event_type_name(EventType t);

struct WatchEvent {
  EventType type;
  std::string kind;
  Value object;
  int64_t revision;
};

struct Key {
  std::string kind, ns, name;
  bool operator<(const Key& o) const { return std::tie(kind, ns, name) < std::tie(o.kind, o.ns, o.name); }
};

class Store {
 public:
  explicit Store(api::Clock clock = api::wall_clock);

  Value create(const std::string& kind, Value obj);
  Value get(const std::string& kind, const std::string& ns, const std::string& name) const;
  bool try_get(const std::string& kind, const std::string& ns, const std::string& name, Value* out) const;
  // ns "" = all namespaces; labels = equality selector; owner = controller-owner index
  std::vector<Value> list(const std::string& kind, const std::string& ns = "",
                          const std::map<std::string, std::string>& labels = {},
                          const std::string& owner = "") const;
  Value update(const std::string& kind, Value obj);         // metadata + spec (+ data)
  Value update_status(const std::string& kind, Value obj);  // status only
  // delete: graceful → set deletionTimestamp and leave removal to `finalize_delete`
  void remove(const std::string& kind, const std::string& ns, const std::string& name, bool graceful = false);
  void finalize_delete(const std::string& kind, const std::string& ns, const std::string& name);

  // watch events (queued; delivered by the caller of drain)
  std::vector<WatchEvent> drain();
  bool has_events() const;
  // block until an event is queued or `timeout_s` passes
  bool wait_events(double timeout_s);
  int64_t revision() const;
  size_t size() const;

  // kinds whose status is a subresource (update() ignores status changes)
  void set_status_subresource(const std::string& kind, bool on);
  // admission of `kind` on create / update / update_status (mutate, or throw
  // ApiError(Invalid)); not applied to mirror_* (server objects are admitted)
  using Admission = std::function<void(Value&)>;
  void set_admission(const std::string& kind, Admission fn);

  // informer-cache mode (k8s backend): store server objects verbatim
  void mirror_put(const std::string& kind, const Value& obj);
  void mirror_delete(const std::string& kind, const std::string& ns, const std::string& name);
  // relist: replace every object of `kind` (in `ns`, "" = all) with `objs`
  void mirror_replace(const std::string& kind, const std::string& ns, const std::vector<Value>& objs);

 private:
  void emit_locked(EventType t, const std::string& kind, const Value& obj);
  void remove_locked(const Key& k);
  void gc_locked(const std::string& uid);
  std::string next_uid_locked();

  api::Clock clock_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<Key, Value> objs_;
  std::map<std::string, bool> status_sub_;
  std::map<std::string, Admission> admission_;
  void admit(const std::string& kind, Value& obj) const;
  std::vector<WatchEvent> pending_;
  int64_t rev_ = 0;
  uint64_t uid_seq_ = 0;
};

// controller owner name of an object if that owner is a PaddleJob
std::string owner_index(const Value& obj);

}  // namespace store
}  // namespace pdo
