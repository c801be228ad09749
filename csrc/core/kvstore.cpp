// SPDX-License-Identifier: Apache-2.0
#include "sync.h"
#include "kvstore.h"

#include <chrono>

namespace pdo {
namespace kv {

std::string KVStore::prefix_end(const std::string& prefix) {
  std::string end = prefix;
  for (int i = (int)end.size() - 1; i >= 0; --i) {
    if ((unsigned char)end[i] < 0xff) {
      end[i] = (char)((unsigned char)end[i] + 1);
      end.resize(i + 1);
      return end;
    }
  }
  return std::string(1, '\0');  // whole keyspace
}

bool KVStore::in_range(const std::string& k, const std::string& key, const std::string& end) const {
  if (end.empty()) return k == key;
  if (end == std::string(1, '\0')) return k >= key;
  return k >= key && k < end;
}

int64_t KVStore::revision() const {
  std::lock_guard<std::mutex> g(mu_);
  return rev_;
}

size_t KVStore::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return data_.size();
}

void KVStore::notify_locked(int64_t rev, const std::vector<Event>& evs) {
  if (evs.empty()) return;
  for (auto& e : evs) history_.emplace_back(rev, e);
  if (history_.size() > 20000) history_.erase(history_.begin(), history_.begin() + 10000);
  std::vector<int64_t> dead;
  for (auto& w : watchers_) {
    std::vector<Event> mine;
    for (auto& e : evs)
      if (in_range(e.kv.key, w.second.key, w.second.end)) mine.push_back(e);
    if (!mine.empty() && !w.second.fn(rev, mine)) dead.push_back(w.first);
  }
  for (auto id : dead) watchers_.erase(id);
  cv_.notify_all();
}

int64_t KVStore::put_locked(const std::string& key, const std::string& value, int64_t lease,
                            std::vector<Event>& evs) {
  Event e;
  e.type = Event::Put;
  auto it = data_.find(key);
  if (it != data_.end()) {
    e.prev = it->second;
    e.has_prev = true;
  }
  KeyValue& kv = data_[key];
  kv.key = key;
  kv.value = value;
  kv.lease = lease;
  kv.mod_revision = rev_;
  if (!e.has_prev) {
    kv.create_revision = rev_;
    kv.version = 1;
  } else {
    kv.version += 1;
  }
  e.kv = kv;
  evs.push_back(e);
  return rev_;
}

int64_t KVStore::put(const std::string& key, const std::string& value, int64_t lease, KeyValue* prev,
                     bool* had_prev) {
  std::lock_guard<std::mutex> g(mu_);
  if (lease && !leases_.count(lease)) return -1;
  std::vector<Event> evs;
  ++rev_;
  put_locked(key, value, lease, evs);
  if (had_prev) *had_prev = evs[0].has_prev;
  if (prev && evs[0].has_prev) *prev = evs[0].prev;
  notify_locked(rev_, evs);
  return rev_;
}

std::vector<KeyValue> KVStore::range_locked(const std::string& key, const std::string& end, int64_t limit,
                                            int64_t* count) const {
  std::vector<KeyValue> out;
  int64_t n = 0;
  if (end.empty()) {
    auto it = data_.find(key);
    if (it != data_.end()) {
      out.push_back(it->second);
      n = 1;
    }
  } else {
    for (auto it = data_.lower_bound(key); it != data_.end(); ++it) {
      if (!in_range(it->first, key, end)) break;
      ++n;
      if (limit <= 0 || (int64_t)out.size() < limit) out.push_back(it->second);
    }
  }
  if (count) *count = n;
  return out;
}

std::vector<KeyValue> KVStore::range(const std::string& key, const std::string& range_end, int64_t limit,
                                     int64_t* count) const {
  std::lock_guard<std::mutex> g(mu_);
  return range_locked(key, range_end, limit, count);
}

bool KVStore::get(const std::string& key, KeyValue* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = data_.find(key);
  if (it == data_.end()) return false;
  if (out) *out = it->second;
  return true;
}

int64_t KVStore::delete_locked(const std::string& key, const std::string& end, std::vector<Event>& evs,
                               std::vector<KeyValue>* prev) {
  std::vector<std::string> victims;
  for (auto& kv : range_locked(key, end, 0, nullptr)) victims.push_back(kv.key);
  for (auto& k : victims) {
    Event e;
    e.type = Event::Delete;
    e.prev = data_[k];
    e.has_prev = true;
    e.kv.key = k;
    e.kv.mod_revision = rev_;
    if (prev) prev->push_back(data_[k]);
    data_.erase(k);
    evs.push_back(e);
  }
  return (int64_t)victims.size();
}

int64_t KVStore::delete_range(const std::string& key, const std::string& range_end, std::vector<KeyValue>* prev) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Event> evs;
  ++rev_;
  int64_t n = delete_locked(key, range_end, evs, prev);
  if (n == 0) {
    --rev_;  // etcd does not bump the revision for a no-op delete
    return 0;
  }
  notify_locked(rev_, evs);
  return n;
}

static bool cmp_num(int64_t a, int64_t b, Compare::Result r) {
  switch (r) {
    case Compare::Equal: return a == b;
    case Compare::Greater: return a > b;
    case Compare::Less: return a < b;
    case Compare::NotEqual: return a != b;
  }
  return false;
}

bool KVStore::txn(const std::vector<Compare>& cmp, const std::vector<Op>& success, const std::vector<Op>& failure,
                  std::vector<OpResult>* results) {
  std::lock_guard<std::mutex> g(mu_);
  bool ok = true;
  for (auto& c : cmp) {
    std::vector<KeyValue> kvs = range_locked(c.key, c.range_end, 0, nullptr);
    if (kvs.empty()) {
      // missing key: version/create/mod/lease compare as 0, value compares as ""
      KeyValue z;
      z.key = c.key;
      kvs.push_back(z);
    }
    for (auto& kv : kvs) {
      bool r;
      switch (c.target) {
        case Compare::Version: r = cmp_num(kv.version, c.num, c.result); break;
        case Compare::Create: r = cmp_num(kv.create_revision, c.num, c.result); break;
        case Compare::Mod: r = cmp_num(kv.mod_revision, c.num, c.result); break;
        case Compare::Lease: r = cmp_num(kv.lease, c.num, c.result); break;
        case Compare::Value: {
          int s = kv.value.compare(c.value);
          r = c.result == Compare::Equal ? s == 0
              : c.result == Compare::Greater ? s > 0
              : c.result == Compare::Less    ? s < 0
                                             : s != 0;
          break;
        }
        default: r = false;
      }
      if (!r) ok = false;
    }
  }
  const std::vector<Op>& ops = ok ? success : failure;
  bool writes = false;
  for (auto& op : ops)
    if (op.type != Op::Range) writes = true;
  if (writes) ++rev_;
  std::vector<Event> evs;
  for (auto& op : ops) {
    OpResult res;
    res.type = op.type;
    if (op.type == Op::Range) {
      res.kvs = range_locked(op.key, op.range_end, op.limit, &res.count);
    } else if (op.type == Op::Put) {
      auto it = data_.find(op.key);
      if (op.prev_kv && it != data_.end()) res.prev_kvs.push_back(it->second);
      put_locked(op.key, op.value, op.lease, evs);
    } else {
      res.deleted = delete_locked(op.key, op.range_end, evs, op.prev_kv ? &res.prev_kvs : nullptr);
    }
    if (results) results->push_back(res);
  }
  if (writes && evs.empty()) --rev_;
  notify_locked(rev_, evs);
  return ok;
}

int64_t KVStore::lease_grant(int64_t ttl_s, int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  if (id == 0) id = ++next_lease_;
  if (leases_.count(id)) return -1;
  leases_[id] = Lease{ttl_s, clock_() + (double)ttl_s};
  return id;
}

bool KVStore::lease_revoke(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  if (!leases_.erase(id)) return false;
  std::vector<std::string> keys;
  for (auto& kv : data_)
    if (kv.second.lease == id) keys.push_back(kv.first);
  if (keys.empty()) return true;
  ++rev_;
  std::vector<Event> evs;
  for (auto& k : keys) delete_locked(k, "", evs, nullptr);
  notify_locked(rev_, evs);
  return true;
}

int64_t KVStore::lease_keepalive(int64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = leases_.find(id);
  if (it == leases_.end()) return -1;
  it->second.expiry = clock_() + (double)it->second.ttl;
  return it->second.ttl;
}

int64_t KVStore::lease_ttl(int64_t id, std::vector<std::string>* keys) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = leases_.find(id);
  if (it == leases_.end()) return -1;
  if (keys)
    for (auto& kv : data_)
      if (kv.second.lease == id) keys->push_back(kv.first);
  double left = it->second.expiry - clock_();
  return left > 0 ? (int64_t)(left + 0.5) : 0;
}

void KVStore::expire_leases() {
  std::vector<int64_t> dead;
  {
    std::lock_guard<std::mutex> g(mu_);
    double now = clock_();
    for (auto& l : leases_)
      if (l.second.expiry <= now) dead.push_back(l.first);
  }
  for (auto id : dead) lease_revoke(id);
}

int64_t KVStore::watch(const std::string& key, const std::string& range_end, int64_t start_rev, WatchFn fn) {
  std::lock_guard<std::mutex> g(mu_);
  int64_t id = next_watch_++;
  if (start_rev > 0 && start_rev <= rev_) {
    // replay history ≥ start_rev
    std::map<int64_t, std::vector<Event>> by_rev;
    for (auto& h : history_)
      if (h.first >= start_rev && in_range(h.second.kv.key, key, range_end)) by_rev[h.first].push_back(h.second);
    for (auto& r : by_rev)
      if (!fn(r.first, r.second)) return id;
  }
  watchers_[id] = Watcher{key, range_end, std::move(fn)};
  return id;
}

void KVStore::cancel(int64_t watch_id) {
  std::lock_guard<std::mutex> g(mu_);
  watchers_.erase(watch_id);
}

int64_t KVStore::wait_revision(int64_t rev, double timeout_s) {
  std::unique_lock<std::mutex> l(mu_);
  wait_for_s(cv_, l, timeout_s, [&] { return rev_ > rev; });
  return rev_;
}

void KVStore::compact(int64_t rev) {
  std::lock_guard<std::mutex> g(mu_);
  compacted_ = rev;
  std::vector<std::pair<int64_t, Event>> keep;
  for (auto& h : history_)
    if (h.first >= rev) keep.push_back(h);
  history_.swap(keep);
}

}  // namespace kv
}  // namespace pdo
