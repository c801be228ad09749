// SPDX-License-Identifier: Apache-2.0
#include "sync.h"
#include "kvclient.h"

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>

#include "base64.h"
#include "json.h"
#include "metrics.h"

namespace pdo {
namespace kv {

using json::Value;

static std::string b64(const std::string& s) { return b64encode(s); }
static std::string unb64(const Value& v) {
  std::string out;
  b64decode(v.as_string(), &out);
  return out;
}
static int64_t i64(const Value& v) {
  if (v.is_string()) return atoll(v.as_string().c_str());
  return v.as_int();
}
static Value s64(int64_t v) { return Value(std::to_string(v)); }

static Value header_rev(int64_t rev) {
  Value h = Value::object();
  h["cluster_id"] = "14841639068965178418";
  h["member_id"] = "10276657743932975437";
  h["revision"] = s64(rev);
  h["raft_term"] = "2";
  return h;
}

static Value header(const KVStore& s) { return header_rev(s.revision()); }

static Value kv_json(const KeyValue& kv, bool keys_only = false) {
  Value o = Value::object();
  o["key"] = b64(kv.key);
  o["create_revision"] = s64(kv.create_revision);
  o["mod_revision"] = s64(kv.mod_revision);
  o["version"] = s64(kv.version);
  if (!keys_only) o["value"] = b64(kv.value);
  if (kv.lease) o["lease"] = s64(kv.lease);
  return o;
}

static Op parse_op(const Value& v, Op::Type t) {
  Op op;
  op.type = t;
  op.key = unb64(v.get("key"));
  op.range_end = unb64(v.get("range_end"));
  op.value = unb64(v.get("value"));
  op.lease = i64(v.get("lease"));
  op.limit = i64(v.get("limit"));
  op.prev_kv = v.get("prev_kv").as_bool();
  return op;
}

static http::Response ok(const Value& v) {
  http::Response r;
  r.body = v.dump();
  return r;
}

static http::Response bad(const std::string& msg, int code = 400) {
  http::Response r;
  r.status = code;
  Value e = Value::object();
  e["error"] = msg;
  e["message"] = msg;
  e["code"] = 3;
  r.body = e.dump();
  return r;
}

void mount_gateway(http::Server& srv, KVStore& s) {
  auto parse = [](const http::Request& q) { return q.body.empty() ? Value::object() : Value::parse(q.body); };

  srv.route("POST", "/v3/kv/range", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    int64_t count = 0;
    auto kvs = s.range(unb64(in.get("key")), unb64(in.get("range_end")), i64(in.get("limit")), &count);
    Value out = Value::object();
    out["header"] = header(s);
    if (!in.get("count_only").as_bool() && !kvs.empty()) {
      Value a = Value::array();
      for (auto& kv : kvs) a.push_back(kv_json(kv, in.get("keys_only").as_bool()));
      out["kvs"] = a;
    }
    if (count) out["count"] = s64(count);
    int64_t lim = i64(in.get("limit"));
    if (lim > 0 && count > lim) out["more"] = true;
    Metrics::global().inc("pdo_kv_requests_total", {{"op", "range"}});
    return ok(out);
  });

  srv.route("POST", "/v3/kv/put", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    KeyValue prev;
    bool had = false;
    int64_t rev = s.put(unb64(in.get("key")), unb64(in.get("value")), i64(in.get("lease")), &prev, &had);
    if (rev < 0) return bad("etcdserver: requested lease not found", 404);
    Value out = Value::object();
    out["header"] = header(s);
    if (in.get("prev_kv").as_bool() && had) out["prev_kv"] = kv_json(prev);
    Metrics::global().inc("pdo_kv_requests_total", {{"op", "put"}});
    return ok(out);
  });

  srv.route("POST", "/v3/kv/deleterange", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    std::vector<KeyValue> prev;
    int64_t n = s.delete_range(unb64(in.get("key")), unb64(in.get("range_end")), &prev);
    Value out = Value::object();
    out["header"] = header(s);
    if (n) out["deleted"] = s64(n);
    if (in.get("prev_kv").as_bool() && !prev.empty()) {
      Value a = Value::array();
      for (auto& kv : prev) a.push_back(kv_json(kv));
      out["prev_kvs"] = a;
    }
    Metrics::global().inc("pdo_kv_requests_total", {{"op", "delete"}});
    return ok(out);
  });

  srv.route("POST", "/v3/kv/txn", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    std::vector<Compare> cmps;
    for (auto& c : in.get("compare").arr()) {
      Compare x;
      x.key = unb64(c.get("key"));
      x.range_end = unb64(c.get("range_end"));
      const std::string t = c.get("target").str("VERSION");
      const std::string r = c.get("result").str("EQUAL");
      x.target = t == "CREATE" ? Compare::Create : t == "MOD" ? Compare::Mod : t == "VALUE" ? Compare::Value
                 : t == "LEASE" ? Compare::Lease : Compare::Version;
      x.result = r == "GREATER" ? Compare::Greater : r == "LESS" ? Compare::Less
                 : r == "NOT_EQUAL" ? Compare::NotEqual : Compare::Equal;
      if (x.target == Compare::Value) x.value = unb64(c.get("value"));
      else if (x.target == Compare::Create) x.num = i64(c.get("create_revision"));
      else if (x.target == Compare::Mod) x.num = i64(c.get("mod_revision"));
      else if (x.target == Compare::Lease) x.num = i64(c.get("lease"));
      else x.num = i64(c.get("version"));
      cmps.push_back(x);
    }
    auto ops = [](const Value& list) {
      std::vector<Op> out;
      for (auto& o : list.arr()) {
        if (o.has("request_put")) out.push_back(parse_op(o.get("request_put"), Op::Put));
        else if (o.has("request_range")) out.push_back(parse_op(o.get("request_range"), Op::Range));
        else if (o.has("request_delete_range")) out.push_back(parse_op(o.get("request_delete_range"), Op::DeleteRange));
      }
      return out;
    };
    std::vector<OpResult> res;
    bool succeeded = s.txn(cmps, ops(in.get("success")), ops(in.get("failure")), &res);
    Value out = Value::object();
    out["header"] = header(s);
    if (succeeded) out["succeeded"] = true;
    Value rs = Value::array();
    for (auto& r : res) {
      Value one = Value::object();
      if (r.type == Op::Range) {
        Value rr = Value::object();
        rr["header"] = header(s);
        Value a = Value::array();
        for (auto& kv : r.kvs) a.push_back(kv_json(kv));
        if (a.size()) rr["kvs"] = a;
        if (r.count) rr["count"] = s64(r.count);
        one["response_range"] = rr;
      } else if (r.type == Op::Put) {
        Value rr = Value::object();
        rr["header"] = header(s);
        if (!r.prev_kvs.empty()) rr["prev_kv"] = kv_json(r.prev_kvs[0]);
        one["response_put"] = rr;
      } else {
        Value rr = Value::object();
        rr["header"] = header(s);
        if (r.deleted) rr["deleted"] = s64(r.deleted);
        one["response_delete_range"] = rr;
      }
      rs.push_back(one);
    }
    if (rs.size()) out["responses"] = rs;
    Metrics::global().inc("pdo_kv_requests_total", {{"op", "txn"}});
    return ok(out);
  });

  srv.route("POST", "/v3/lease/grant", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    int64_t ttl = i64(in.get("TTL"));
    int64_t id = s.lease_grant(ttl, i64(in.get("ID")));
    if (id < 0) return bad("etcdserver: lease already exists");
    Value out = Value::object();
    out["header"] = header(s);
    out["ID"] = s64(id);
    out["TTL"] = s64(ttl);
    return ok(out);
  });
  srv.route("POST", "/v3/lease/revoke", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    if (!s.lease_revoke(i64(in.get("ID")))) return bad("etcdserver: requested lease not found", 404);
    Value out = Value::object();
    out["header"] = header(s);
    return ok(out);
  });
  srv.route("POST", "/v3/lease/keepalive", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    int64_t ttl = s.lease_keepalive(i64(in.get("ID")));
    Value r = Value::object();
    r["header"] = header(s);
    r["ID"] = s64(i64(in.get("ID")));
    if (ttl >= 0) r["TTL"] = s64(ttl);
    Value out = Value::object();
    out["result"] = r;
    return ok(out);
  });
  srv.route("POST", "/v3/lease/timetolive", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    std::vector<std::string> keys;
    int64_t ttl = s.lease_ttl(i64(in.get("ID")), in.get("keys").as_bool() ? &keys : nullptr);
    Value out = Value::object();
    out["header"] = header(s);
    out["ID"] = s64(i64(in.get("ID")));
    out["TTL"] = s64(ttl);
    if (!keys.empty()) {
      Value a = Value::array();
      for (auto& k : keys) a.push_back(b64(k));
      out["keys"] = a;
    }
    return ok(out);
  });

  srv.route("POST", "/v3/watch", [&s, parse](const http::Request& q) {
    Value in = parse(q);
    const Value& cr = in.get("create_request");
    std::string key = unb64(cr.get("key")), end = unb64(cr.get("range_end"));
    int64_t start = i64(cr.get("start_revision"));
    http::Response r;
    KVStore* sp = &s;
    r.stream = [sp, key, end, start](http::StreamWriter& w) {
      struct Q {
        std::mutex mu;
        std::condition_variable cv;
        std::deque<std::string> lines;
        bool dead = false;
      };
      auto qq = std::make_shared<Q>();
      Value created = Value::object();
      created["result"]["header"] = header(*sp);
      created["result"]["created"] = true;
      // runs under the store lock: must not call back into the store
      int64_t wid = sp->watch(key, end, start, [qq](int64_t rev, const std::vector<Event>& evs) {
        Value res = Value::object();
        Value& rr = res["result"];
        rr["header"] = header_rev(rev);
        Value a = Value::array();
        for (auto& e : evs) {
          Value ev = Value::object();
          if (e.type == Event::Delete) ev["type"] = "DELETE";
          ev["kv"] = kv_json(e.kv);
          if (e.has_prev) ev["prev_kv"] = kv_json(e.prev);
          a.push_back(ev);
        }
        rr["events"] = a;
        std::lock_guard<std::mutex> g(qq->mu);
        if (qq->dead) return false;
        qq->lines.push_back(res.dump() + "\n");
        qq->cv.notify_all();
        return true;
      });
      created["result"]["watch_id"] = s64(wid);
      if (!w.write(created.dump() + "\n")) {
        sp->cancel(wid);
        return;
      }
      while (true) {
        std::deque<std::string> batch;
        {
          std::unique_lock<std::mutex> l(qq->mu);
          wait_for_s(qq->cv, l, 0.5, [&] { return !qq->lines.empty(); });
          batch.swap(qq->lines);
        }
        bool alive = true;
        for (auto& line : batch)
          if (!w.write(line)) alive = false;
        if (!alive || w.closed()) break;
      }
      {
        std::lock_guard<std::mutex> g(qq->mu);
        qq->dead = true;
      }
      sp->cancel(wid);
    };
    return r;
  });

  srv.route("GET", "/health", [](const http::Request&) {
    http::Response r;
    r.body = "{\"health\":\"true\",\"reason\":\"\"}";
    return r;
  });
  srv.route("GET", "/version", [](const http::Request&) {
    http::Response r;
    r.body = "{\"etcdserver\":\"3.5.0-pdo\",\"etcdcluster\":\"3.5.0\"}";
    return r;
  });
}

// ------------------------------------------------------------------ clients
bool LocalClient::get(const std::string& key, std::vector<KeyValue>* kvs) {
  *kvs = s_->range(key);
  return true;
}

bool LocalClient::put(const std::string& key, const std::string& value) { return s_->put(key, value) > 0; }

HttpClient::HttpClient(const std::string& endpoints, double timeout_s) : timeout_(timeout_s) {
  size_t pos = 0;
  while (pos <= endpoints.size()) {
    size_t c = endpoints.find(',', pos);
    std::string e = endpoints.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    if (!e.empty()) eps_.push_back(e);
    if (c == std::string::npos) break;
    pos = c + 1;
  }
}

bool HttpClient::call(const std::string& path, const std::string& body, std::string* out) {
  http::ClientOptions opt;
  opt.timeout_s = timeout_;
  for (auto& e : eps_) {
    std::string url = e.find("://") == std::string::npos ? "http://" + e + path : e + path;
    auto r = http::request("POST", url, body, opt);
    if (r.status == 200) {
      *out = r.body;
      return true;
    }
  }
  return false;
}

bool HttpClient::get(const std::string& key, std::vector<KeyValue>* kvs) {
  Value in = Value::object();
  in["key"] = b64(key);
  std::string body;
  if (!call("/v3/kv/range", in.dump(), &body)) return false;
  Value out = Value::parse(body);
  kvs->clear();
  for (auto& k : out.get("kvs").arr()) {
    KeyValue kv;
    kv.key = unb64(k.get("key"));
    kv.value = unb64(k.get("value"));
    kv.create_revision = i64(k.get("create_revision"));
    kv.mod_revision = i64(k.get("mod_revision"));
    kv.version = i64(k.get("version"));
    kv.lease = i64(k.get("lease"));
    kvs->push_back(kv);
  }
  return true;
}

bool HttpClient::put(const std::string& key, const std::string& value) {
  Value in = Value::object();
  in["key"] = b64(key);
  in["value"] = b64(value);
  std::string body;
  return call("/v3/kv/put", in.dump(), &body);
}

}  // namespace kv
}  // namespace pdo
