// SPDX-License-Identifier: Apache-2.0
// pdo-kv: an etcd-v3-subset key/value store (MVCC revisions, range/prefix
// reads, transactions with compare-and-swap, leases with TTL, watches with
// history replay).
//
// Replaces the external etcd of the reference's elastic mode
// (deploy/elastic/etcd.yaml; controllers/paddlejob_elastic.go:27-55 uses
// Get/Put on /paddle/<ns>-<name>/np) and serves the launcher's rendezvous
// (RCCL unique-id exchange, readiness barrier, elastic membership).  The
// HTTP front end (kvserver) speaks etcd's grpc-gateway JSON API, so etcd
// clients using the JSON gateway and pdo's clients are interchangeable.
#pragma once

#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "api.h"

namespace pdo {
namespace kv {

struct KeyValue {
  std::string key, value;
  int64_t create_revision = 0, mod_revision = 0, version = 0, lease = 0;
};

struct Event {
  enum Type { Put, Delete } type;
  KeyValue kv;
  KeyValue prev;
  bool has_prev = false;
};

struct Compare {
  enum Target { Version, Create, Mod, Value, Lease } target = Version;
  enum Result { Equal, Greater, Less, NotEqual } result = Equal;
  std::string key, range_end;
  int64_t num = 0;
  std::string value;
};

struct Op {
  enum Type { Range, Put, DeleteRange } type = Range;
  std::string key, range_end, value;
  int64_t lease = 0, limit = 0;
  bool prev_kv = false;
};

struct OpResult {
  Op::Type type;
  std::vector<KeyValue> kvs;
  int64_t count = 0;
  int64_t deleted = 0;
  std::vector<KeyValue> prev_kvs;
};

using WatchFn = std::function<bool(int64_t revision, const std::vector<Event>&)>;  // false → cancel

class KVStore {
 public:
  explicit KVStore(api::Clock clock = api::wall_clock) : clock_(std::move(clock)) {}

  int64_t revision() const;
  int64_t put(const std::string& key, const std::string& value, int64_t lease = 0, KeyValue* prev = nullptr,
              bool* had_prev = nullptr);
  std::vector<KeyValue> range(const std::string& key, const std::string& range_end = "", int64_t limit = 0,
                              int64_t* count = nullptr) const;
  bool get(const std::string& key, KeyValue* out) const;
  int64_t delete_range(const std::string& key, const std::string& range_end = "",
                       std::vector<KeyValue>* prev = nullptr);
  bool txn(const std::vector<Compare>& cmp, const std::vector<Op>& success, const std::vector<Op>& failure,
           std::vector<OpResult>* results);

  int64_t lease_grant(int64_t ttl_s, int64_t id = 0);
  bool lease_revoke(int64_t id);
  int64_t lease_keepalive(int64_t id);  // remaining TTL (s) or -1
  int64_t lease_ttl(int64_t id, std::vector<std::string>* keys = nullptr) const;
  void expire_leases();  // called periodically

  // watch [key, range_end) from start_rev (0 = now); returns id
  int64_t watch(const std::string& key, const std::string& range_end, int64_t start_rev, WatchFn fn);
  void cancel(int64_t watch_id);
  // block until revision > rev or timeout; returns current revision
  int64_t wait_revision(int64_t rev, double timeout_s);
  void compact(int64_t rev);
  size_t size() const;

  static std::string prefix_end(const std::string& prefix);  // etcd clientv3.GetPrefixRangeEnd

 private:
  bool in_range(const std::string& k, const std::string& key, const std::string& end) const;
  int64_t put_locked(const std::string& key, const std::string& value, int64_t lease, std::vector<Event>& evs);
  int64_t delete_locked(const std::string& key, const std::string& range_end, std::vector<Event>& evs,
                        std::vector<KeyValue>* prev);
  std::vector<KeyValue> range_locked(const std::string& key, const std::string& range_end, int64_t limit,
                                     int64_t* count) const;
  void notify_locked(int64_t rev, const std::vector<Event>& evs);

  struct Lease {
    int64_t ttl;
    double expiry;
  };
  struct Watcher {
    std::string key, end;
    WatchFn fn;
  };
  api::Clock clock_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, KeyValue> data_;
  std::map<int64_t, Lease> leases_;
  std::map<int64_t, Watcher> watchers_;
  std::vector<std::pair<int64_t, Event>> history_;  // for start_revision replay
  int64_t rev_ = 1;
  int64_t next_lease_ = 0x7ab10000;
  int64_t next_watch_ = 1;
  int64_t compacted_ = 0;
};

// JSON gateway mounted on an http::Server (see kvserver.cpp for routes)
namespace http_api {
class Server;
}

}  // namespace kv
}  // namespace pdo
