// SPDX-License-Identifier: Apache-2.0
#include "sync.h"
#include "store.h"

#include "schema.h"

#include <chrono>
#include <cstdio>
#include <random>

#include "builders.h"

namespace pdo {
namespace store {

const char* event_type_name(EventType t) {
  switch (t) {
    case EventType::Added: return "ADDED";
    case EventType::Modified: return "MODIFIED";
    case EventType::Deleted: return "DELETED";
  }
  return "?";
}

std::string owner_index(const Value& obj) { return build::controller_owner(obj); }

Store::Store(api::Clock clock) : clock_(std::move(clock)) {
  status_sub_[api::kKind] = true;  // +kubebuilder:subresource:status
  status_sub_["Pod"] = true;
  status_sub_["PodGroup"] = true;
  // the PaddleJob CRD's structural schema: pruning + validation on write
  admission_[api::kKind] = schema::admit_paddlejob;
}

void Store::set_status_subresource(const std::string& kind, bool on) {
  std::lock_guard<std::mutex> g(mu_);
  status_sub_[kind] = on;
}

std::string Store::next_uid_locked() {
  static std::mt19937_64 rng(std::random_device{}());
  uint64_t a = rng(), b = rng() ^ (++uid_seq_);
  char buf[40];
  snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xffff),
           (unsigned)(0x4000 | (a & 0x0fff)), (unsigned)(0x8000 | ((b >> 48) & 0x3fff)),
           (unsigned long long)(b & 0xffffffffffffULL));
  return buf;
}

static Key key_of(const std::string& kind, const Value& obj) {
  return Key{kind, obj.at_path("metadata.namespace").str(), obj.at_path("metadata.name").str()};
}

void Store::emit_locked(EventType t, const std::string& kind, const Value& obj) {
  pending_.push_back(WatchEvent{t, kind, obj, rev_});
  cv_.notify_all();
}

void Store::set_admission(const std::string& kind, Admission fn) {
  std::lock_guard<std::mutex> g(mu_);
  admission_[kind] = std::move(fn);
}

void Store::admit(const std::string& kind, Value& obj) const {
  Admission fn;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = admission_.find(kind);
    if (it == admission_.end()) return;
    fn = it->second;
  }
  fn(obj);
}

Value Store::create(const std::string& kind, Value obj) {
  admit(kind, obj);
  std::lock_guard<std::mutex> g(mu_);
  Key k = key_of(kind, obj);
  if (k.name.empty()) {
    const std::string gen = obj.at_path("metadata.generateName").str();
    if (gen.empty()) throw ApiError(ApiError::Invalid, kind + ": metadata.name is required");
    k.name = gen + next_uid_locked().substr(0, 5);
    obj["metadata"]["name"] = k.name;
  }
  if (objs_.count(k)) throw ApiError(ApiError::AlreadyExists, kind + " \"" + k.name + "\" already exists");
  Value& md = obj["metadata"];
  md["uid"] = next_uid_locked();
  md["resourceVersion"] = std::to_string(++rev_);
  md["creationTimestamp"] = api::rfc3339(clock_());
  md["generation"] = 1;
  md.erase("deletionTimestamp");
  objs_[k] = obj;
  emit_locked(EventType::Added, kind, obj);
  return obj;
}

Value Store::get(const std::string& kind, const std::string& ns, const std::string& name) const {
  Value out;
  if (!try_get(kind, ns, name, &out))
    throw ApiError(ApiError::NotFound, kind + " \"" + ns + "/" + name + "\" not found");
  return out;
}

bool Store::try_get(const std::string& kind, const std::string& ns, const std::string& name, Value* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(Key{kind, ns, name});
  if (it == objs_.end()) return false;
  if (out) *out = it->second;
  return true;
}

std::vector<Value> Store::list(const std::string& kind, const std::string& ns,
                               const std::map<std::string, std::string>& labels, const std::string& owner) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Value> out;
  auto it = objs_.lower_bound(Key{kind, ns, ""});
  for (; it != objs_.end() && it->first.kind == kind; ++it) {
    if (!ns.empty() && it->first.ns != ns) break;
    const Value& o = it->second;
    bool ok = true;
    for (auto& l : labels)
      if (o.at_path("metadata.labels").get(l.first).as_string() != l.second) {
        ok = false;
        break;
      }
    if (ok && !owner.empty() && owner_index(o) != owner) ok = false;
    if (ok) out.push_back(o);
  }
  return out;
}

Value Store::update(const std::string& kind, Value obj) {
  admit(kind, obj);
  std::lock_guard<std::mutex> g(mu_);
  Key k = key_of(kind, obj);
  auto it = objs_.find(k);
  if (it == objs_.end()) throw ApiError(ApiError::NotFound, kind + " \"" + k.name + "\" not found");
  Value& cur = it->second;
  const std::string rv = obj.at_path("metadata.resourceVersion").str();
  if (!rv.empty() && rv != cur.at_path("metadata.resourceVersion").as_string())
    throw ApiError(ApiError::Conflict, "Operation cannot be fulfilled on " + kind + " \"" + k.name +
                                           "\": the object has been modified; please apply your changes to the "
                                           "latest version and try again");
  Value next = obj;
  // immutable / server-owned metadata
  for (const char* f : {"uid", "creationTimestamp", "generation", "deletionTimestamp"}) {
    const Value& v = cur.at_path(std::string("metadata.") + f);
    if (v.is_null()) next["metadata"].erase(f);
    else next["metadata"][f] = v;
  }
  if (status_sub_[kind]) {
    const Value& st = cur.get("status");
    if (st.is_null()) next.erase("status");
    else next["status"] = st;
  }
  if (!(next.get("spec") == cur.get("spec")))
    next["metadata"]["generation"] = cur.at_path("metadata.generation").as_int(1) + 1;
  // a deleting object whose last finalizer is removed goes away now
  const bool deleting = !cur.at_path("metadata.deletionTimestamp").is_null();
  if (next == cur) return cur;  // no-op update: no new revision (apiserver behaviour)
  next["metadata"]["resourceVersion"] = std::to_string(++rev_);
  cur = next;
  if (deleting && cur.at_path("metadata.finalizers").size() == 0) {
    Value gone = cur;
    remove_locked(k);
    return gone;
  }
  emit_locked(EventType::Modified, kind, cur);
  return cur;
}

Value Store::update_status(const std::string& kind, Value obj) {
  std::lock_guard<std::mutex> g(mu_);
  Key k = key_of(kind, obj);
  auto it = objs_.find(k);
  if (it == objs_.end()) throw ApiError(ApiError::NotFound, kind + " \"" + k.name + "\" not found");
  Value& cur = it->second;
  const std::string rv = obj.at_path("metadata.resourceVersion").str();
  if (!rv.empty() && rv != cur.at_path("metadata.resourceVersion").as_string())
    throw ApiError(ApiError::Conflict, "Operation cannot be fulfilled on " + kind + " \"" + k.name +
                                           "\": the object has been modified");
  if (obj.get("status") == cur.get("status")) return cur;
  cur["status"] = obj.get("status");
  cur["metadata"]["resourceVersion"] = std::to_string(++rev_);
  emit_locked(EventType::Modified, kind, cur);
  return cur;
}

void Store::remove_locked(const Key& k) {
  auto it = objs_.find(k);
  if (it == objs_.end()) return;
  Value gone = it->second;
  objs_.erase(it);
  ++rev_;
  gone["metadata"]["resourceVersion"] = std::to_string(rev_);
  emit_locked(EventType::Deleted, k.kind, gone);
  const std::string uid = gone.at_path("metadata.uid").str();
  if (!uid.empty()) gc_locked(uid);
}

void Store::gc_locked(const std::string& uid) {
  // background propagation: dependents of a removed owner are deleted
  std::vector<Key> victims;
  for (auto& kv : objs_) {
    for (auto& r : kv.second.at_path("metadata.ownerReferences").arr())
      if (r.get("uid").as_string() == uid) {
        victims.push_back(kv.first);
        break;
      }
  }
  for (auto& k : victims) {
    auto it = objs_.find(k);
    if (it == objs_.end()) continue;
    Value& o = it->second;
    if (o.at_path("metadata.finalizers").size() > 0 || (k.kind == "Pod" && o.at_path("spec.nodeName").is_string())) {
      if (o.at_path("metadata.deletionTimestamp").is_null()) {
        o["metadata"]["deletionTimestamp"] = api::rfc3339(clock_());
        o["metadata"]["resourceVersion"] = std::to_string(++rev_);
        emit_locked(EventType::Modified, k.kind, o);
      }
    } else {
      remove_locked(k);
    }
  }
}

void Store::remove(const std::string& kind, const std::string& ns, const std::string& name, bool graceful) {
  std::lock_guard<std::mutex> g(mu_);
  Key k{kind, ns, name};
  auto it = objs_.find(k);
  if (it == objs_.end()) throw ApiError(ApiError::NotFound, kind + " \"" + ns + "/" + name + "\" not found");
  Value& o = it->second;
  if (!o.at_path("metadata.deletionTimestamp").is_null()) {
    // already terminating: a non-graceful delete (grace period 0) finalizes it
    if (!graceful && o.at_path("metadata.finalizers").size() == 0) remove_locked(k);
    return;
  }
  const bool has_fin = o.at_path("metadata.finalizers").size() > 0;
  if (has_fin || graceful) {
    o["metadata"]["deletionTimestamp"] = api::rfc3339(clock_());
    o["metadata"]["resourceVersion"] = std::to_string(++rev_);
    emit_locked(EventType::Modified, kind, o);
    return;
  }
  remove_locked(k);
}

void Store::finalize_delete(const std::string& kind, const std::string& ns, const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  remove_locked(Key{kind, ns, name});
}

void Store::mirror_put(const std::string& kind, const Value& obj) {
  std::lock_guard<std::mutex> g(mu_);
  Key k = key_of(kind, obj);
  auto it = objs_.find(k);
  const bool existed = it != objs_.end();
  if (existed && it->second.at_path("metadata.resourceVersion") == obj.at_path("metadata.resourceVersion")) return;
  objs_[k] = obj;
  ++rev_;
  emit_locked(existed ? EventType::Modified : EventType::Added, kind, obj);
}

void Store::mirror_delete(const std::string& kind, const std::string& ns, const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = objs_.find(Key{kind, ns, name});
  if (it == objs_.end()) return;
  Value gone = it->second;
  objs_.erase(it);
  ++rev_;
  emit_locked(EventType::Deleted, kind, gone);
}

void Store::mirror_replace(const std::string& kind, const std::string& ns, const std::vector<Value>& objs) {
  std::map<Key, Value> fresh;
  for (auto& o : objs) fresh[key_of(kind, o)] = o;
  std::vector<Key> stale;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : objs_)
      if (kv.first.kind == kind && (ns.empty() || kv.first.ns == ns) && !fresh.count(kv.first))
        stale.push_back(kv.first);
  }
  for (auto& k : stale) mirror_delete(kind, k.ns, k.name);
  for (auto& kv : fresh) mirror_put(kind, kv.second);
}

std::vector<WatchEvent> Store::drain() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<WatchEvent> out;
  out.swap(pending_);
  return out;
}

bool Store::has_events() const {
  std::lock_guard<std::mutex> g(mu_);
  return !pending_.empty();
}

bool Store::wait_events(double timeout_s) {
  std::unique_lock<std::mutex> l(mu_);
  if (!pending_.empty()) return true;
  wait_for_s(cv_, l, timeout_s, [&] { return !pending_.empty(); });
  return !pending_.empty();
}

int64_t Store::revision() const {
  std::lock_guard<std::mutex> g(mu_);
  return rev_;
}

size_t Store::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return objs_.size();
}

}  // namespace store
}  // namespace pdo
