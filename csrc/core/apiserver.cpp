// SPDX-License-Identifier: Apache-2.0
#include "sync.h"
#include "apiserver.h"

#include <fstream>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <sstream>

#include "cluster.h"
#include "metrics.h"

namespace pdo {

using json::Value;

const std::vector<KindInfo>& known_kinds() {
  static const std::vector<KindInfo> k = {
      {"Pod", "v1", "pods", true},
      {"Service", "v1", "services", true},
      {"ConfigMap", "v1", "configmaps", true},
      {"Event", "v1", "events", true},
      {"PaddleJob", "batch.paddlepaddle.org/v1", "paddlejobs", true},
      {"PodGroup", "scheduling.volcano.sh/v1beta1", "podgroups", true},
      {"Lease", "coordination.k8s.io/v1", "leases", true},
  };
  return k;
}

const KindInfo* kind_by_plural(const std::string& plural) {
  for (auto& k : known_kinds())
    if (k.plural == plural) return &k;
  return nullptr;
}

const KindInfo* kind_by_name(const std::string& kind) {
  for (auto& k : known_kinds())
    if (k.kind == kind) return &k;
  return nullptr;
}

std::string collection_path(const KindInfo& k, const std::string& ns) {
  const std::string base = k.group_version == "v1" ? "/api/v1" : "/apis/" + k.group_version;
  return ns.empty() ? base + "/" + k.plural : base + "/namespaces/" + ns + "/" + k.plural;
}

int WatchHub::subscribe(std::function<bool(const store::WatchEvent&)> fn) {
  std::lock_guard<std::mutex> g(mu_);
  subs_[next_] = std::move(fn);
  return next_++;
}

void WatchHub::unsubscribe(int id) {
  std::lock_guard<std::mutex> g(mu_);
  subs_.erase(id);
}

void WatchHub::publish(const store::WatchEvent& ev) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = subs_.begin(); it != subs_.end();) {
    if (!it->second(ev)) it = subs_.erase(it);
    else ++it;
  }
}

static http::Response status_resp(int code, const std::string& reason, const std::string& msg) {
  http::Response r;
  r.status = code;
  Value s = Value::object();
  s["kind"] = "Status";
  s["apiVersion"] = "v1";
  s["metadata"] = Value::object();
  s["status"] = "Failure";
  s["message"] = msg;
  s["reason"] = reason;
  s["code"] = code;
  r.body = s.dump();
  return r;
}

static std::string lower_ascii(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

static http::Response api_error(const store::ApiError& e) {
  switch (e.code) {
    case store::ApiError::NotFound: return status_resp(404, "NotFound", e.what());
    case store::ApiError::AlreadyExists: return status_resp(409, "AlreadyExists", e.what());
    case store::ApiError::Conflict: return status_resp(409, "Conflict", e.what());
    default: return status_resp(422, "Invalid", e.what());
  }
}

static std::map<std::string, std::string> parse_selector(const std::string& sel) {
  std::map<std::string, std::string> out;
  std::stringstream ss(sel);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    size_t eq = tok.find('=');
    if (eq == std::string::npos) continue;
    std::string k = tok.substr(0, eq), v = tok.substr(eq + 1);
    if (!v.empty() && v[0] == '=') v = v.substr(1);
    out[k] = v;
  }
  return out;
}

static bool label_match(const Value& obj, const std::map<std::string, std::string>& sel) {
  for (auto& kv : sel)
    if (obj.at_path("metadata.labels").get(kv.first).as_string() != kv.second) return false;
  return true;
}

// parse /api/v1/... or /apis/<g>/<v>/... into (kind, ns, name, sub)
static bool parse_path(const std::string& path, const KindInfo** kind, std::string* ns, std::string* name,
                       std::string* sub) {
  std::vector<std::string> seg;
  std::stringstream ss(path);
  std::string s;
  while (std::getline(ss, s, '/'))
    if (!s.empty()) seg.push_back(s);
  size_t i;
  if (seg.size() >= 2 && seg[0] == "api" && seg[1] == "v1") i = 2;
  else if (seg.size() >= 3 && seg[0] == "apis") i = 3;
  else return false;
  if (i < seg.size() && seg[i] == "namespaces" && i + 2 < seg.size() + 0 && i + 1 < seg.size()) {
    if (i + 2 >= seg.size()) return false;  // /namespaces/{ns} itself: not served
    *ns = seg[i + 1];
    i += 2;
  }
  if (i >= seg.size()) return false;
  *kind = kind_by_plural(seg[i]);
  if (!*kind) return false;
  if (i + 1 < seg.size()) *name = seg[i + 1];
  if (i + 2 < seg.size()) *sub = seg[i + 2];
  return true;
}

void mount_apiserver(http::Server& srv, store::Store& st, WatchHub& hub, Cluster* cluster) {
  auto handler = [&st, &hub, cluster](const http::Request& q) -> http::Response {
    const KindInfo* k = nullptr;
    std::string ns, name, sub;
    if (!parse_path(q.path, &k, &ns, &name, &sub)) return status_resp(404, "NotFound", "unknown path " + q.path);
    Metrics::global().inc("apiserver_request_total", {{"verb", q.method}, {"resource", k->plural}});
    try {
      if (q.method == "GET" && name.empty()) {
        auto sel = parse_selector(q.param("labelSelector"));
        if (q.param("watch") == "true" || q.param("watch") == "1") {
          http::Response r;
          const std::string kind = k->kind;
          std::vector<Value> initial;
          if (q.param("resourceVersion").empty() || q.param("sendInitialEvents") == "true")
            initial = st.list(kind, ns, sel);
          WatchHub* hp = &hub;
          r.stream = [hp, kind, ns, sel, initial](http::StreamWriter& w) {
            struct Q {
              std::mutex mu;
              std::condition_variable cv;
              std::deque<std::string> lines;
              bool dead = false;
            };
            auto qq = std::make_shared<Q>();
            int id = hp->subscribe([qq, kind, ns, sel](const store::WatchEvent& ev) {
              if (ev.kind != kind) return true;
              if (!ns.empty() && ev.object.at_path("metadata.namespace").as_string() != ns) return true;
              if (!label_match(ev.object, sel)) return true;
              Value line = Value::object();
              line["type"] = store::event_type_name(ev.type);
              line["object"] = ev.object;
              std::lock_guard<std::mutex> g(qq->mu);
              if (qq->dead) return false;
              qq->lines.push_back(line.dump() + "\n");
              qq->cv.notify_all();
              return true;
            });
            bool alive = true;
            for (auto& o : initial) {
              Value line = Value::object();
              line["type"] = "ADDED";
              line["object"] = o;
              if (!w.write(line.dump() + "\n")) alive = false;
            }
            while (alive) {
              std::deque<std::string> batch;
              {
                std::unique_lock<std::mutex> l(qq->mu);
                wait_for_s(qq->cv, l, 0.5, [&] { return !qq->lines.empty(); });
                batch.swap(qq->lines);
              }
              for (auto& line : batch)
                if (!w.write(line)) alive = false;
              if (w.closed()) alive = false;
            }
            {
              std::lock_guard<std::mutex> g(qq->mu);
              qq->dead = true;
            }
            hp->unsubscribe(id);
          };
          return r;
        }
        Value list = Value::object();
        list["apiVersion"] = k->group_version;
        list["kind"] = k->kind + "List";
        list["metadata"]["resourceVersion"] = std::to_string(st.revision());
        Value items = Value::array();
        for (auto& o : st.list(k->kind, ns, sel)) items.push_back(o);
        list["items"] = items;
        http::Response r;
        r.body = list.dump();
        return r;
      }
      if ((q.method == "GET" || q.method == "POST") && sub == "exec" && k->kind == "Pod") {
        // kubectl exec / the k8s-backend coordinator: WebSocket upgrade with the
        // channel.k8s.io protocols (kube-apiserver also accepts SPDY; pdo speaks
        // only WebSocket).  Frames: [channel byte][data]; channel 3 = Status.
        st.get(k->kind, ns, name);  // 404 if the pod does not exist
        if (lower_ascii(q.headers.count("upgrade") ? q.headers.at("upgrade") : "") != "websocket" ||
            !q.headers.count("sec-websocket-key"))
          return status_resp(400, "BadRequest", "pods/exec requires a WebSocket upgrade (v4/v5.channel.k8s.io)");
        std::string proto;
        const std::string offered = q.headers.count("sec-websocket-protocol") ? q.headers.at("sec-websocket-protocol") : "";
        for (const char* p : {"v5.channel.k8s.io", "v4.channel.k8s.io", "channel.k8s.io"})
          if (offered.find(p) != std::string::npos) {
            proto = p;
            break;
          }
        if (proto.empty()) return status_resp(400, "BadRequest", "no supported exec subprotocol offered");
        const std::vector<std::string> argv = q.params("command");
        if (argv.empty()) return status_resp(400, "BadRequest", "you must specify at least 1 command");
        const std::string container = q.param("container");
        http::Response r;
        r.status = 101;
        r.headers["Upgrade"] = "websocket";
        r.headers["Connection"] = "Upgrade";
        r.headers["Sec-WebSocket-Accept"] = http::ws_accept_key(q.headers.at("sec-websocket-key"));
        r.headers["Sec-WebSocket-Protocol"] = proto;
        r.upgrade = [cluster, ns, name, container, argv](int fd) {
          http::WsConn ws(fd);
          const bool ok = cluster && cluster->exec(ns, name, container, argv);
          Value s = Value::object();
          s["metadata"] = Value::object();
          if (ok) {
            s["status"] = "Success";
          } else {
            s["status"] = "Failure";
            s["message"] = "command terminated with non-zero exit code";
            s["reason"] = "NonZeroExitCode";
            Value cause = Value::object();
            cause["reason"] = "ExitCode";
            cause["message"] = "1";
            s["details"]["causes"] = Value::array();
            s["details"]["causes"].push_back(cause);
          }
          ws.send(http::kWsBinary, std::string(1, '\x03') + s.dump());
          ws.send(http::kWsClose, std::string("\x03\xe8", 2));
          int op;
          std::string msg;
          ws.recv(&op, &msg, 1.0);  // the client's close, if it sends one
        };
        return r;
      }
      if (q.method == "GET" && sub == "log" && k->kind == "Pod") {
        // kubectl logs: local backend reads the container log from the agent's sandbox
        st.get(k->kind, ns, name);  // 404 if the pod does not exist
        Agent* a = cluster ? cluster->agent_for(ns, name) : nullptr;
        std::string dir = a ? a->sandbox_of(ns, name) : "";
        if (dir.empty()) return status_resp(404, "NotFound", "no log for pod " + name);
        std::string c = q.param("container");
        if (c.empty()) c = st.get(k->kind, ns, name).at_path("spec.containers").arr().front().get("name").str();
        std::ifstream f(dir + "/" + c + ".log", std::ios::binary);
        std::stringstream buf;
        buf << f.rdbuf();
        std::string body = buf.str();
        const std::string tb = q.param("limitBytes");
        if (!tb.empty() && (size_t)atoll(tb.c_str()) < body.size()) body = body.substr(body.size() - atoll(tb.c_str()));
        http::Response r;
        r.content_type = "text/plain";
        r.body = body;
        return r;
      }
      if (q.method == "GET") {
        http::Response r;
        r.body = st.get(k->kind, ns, name).dump();
        return r;
      }
      if (q.method == "POST" && name.empty()) {
        Value obj = Value::parse(q.body);
        if (!ns.empty()) obj["metadata"]["namespace"] = ns;
        api::set_type_meta(obj, k->group_version, k->kind);
        http::Response r;
        r.status = 201;
        r.body = st.create(k->kind, obj).dump();
        return r;
      }
      if ((q.method == "PUT" || q.method == "PATCH") && !name.empty()) {
        Value obj = Value::parse(q.body);
        obj["metadata"]["namespace"] = ns;
        obj["metadata"]["name"] = name;
        if (q.method == "PATCH") {
          // merge patch (RFC 7386) onto the current object
          Value cur = st.get(k->kind, ns, name);
          std::function<void(Value&, const Value&)> merge = [&](Value& dst, const Value& p) {
            if (!p.is_object()) {
              dst = p;
              return;
            }
            if (!dst.is_object()) dst = Value::object();
            for (auto& m : p.obj()) {
              if (m.second.is_null()) dst.erase(m.first);
              else merge(dst[m.first], m.second);
            }
          };
          merge(cur, obj);
          obj = cur;
        }
        http::Response r;
        r.body = (sub == "status" ? st.update_status(k->kind, obj) : st.update(k->kind, obj)).dump();
        return r;
      }
      if (q.method == "DELETE" && !name.empty()) {
        Value cur = st.get(k->kind, ns, name);
        const bool graceful = k->kind == "Pod" && cur.at_path("spec.nodeName").is_string();
        st.remove(k->kind, ns, name, graceful);
        http::Response r;
        Value s = Value::object();
        s["kind"] = "Status";
        s["apiVersion"] = "v1";
        s["status"] = "Success";
        s["details"]["name"] = name;
        s["details"]["kind"] = k->plural;
        r.body = s.dump();
        return r;
      }
      return status_resp(405, "MethodNotAllowed", q.method + " " + q.path);
    } catch (const store::ApiError& e) {
      return api_error(e);
    } catch (const json::ParseError& e) {
      return status_resp(400, "BadRequest", e.what());
    }
  };
  srv.route("*", "/api/v1/*", handler);
  srv.route("*", "/apis/*", handler);
  srv.route("GET", "/version", [](const http::Request&) {
    http::Response r;
    r.body = "{\"major\":\"1\",\"minor\":\"22\",\"gitVersion\":\"v1.22.0-pdo-local\",\"platform\":\"linux/amd64\"}";
    return r;
  });
  srv.route("GET", "/api", [](const http::Request&) {
    http::Response r;
    r.body = "{\"kind\":\"APIVersions\",\"versions\":[\"v1\"]}";
    return r;
  });
  if (cluster) {
    srv.route("POST", "/pdo/v1/namespaces/*", [cluster](const http::Request& q) -> http::Response {
      // /pdo/v1/namespaces/{ns}/pods/{name}/{exec|kill}
      std::vector<std::string> seg;
      std::stringstream ss(q.path);
      std::string s;
      while (std::getline(ss, s, '/'))
        if (!s.empty()) seg.push_back(s);
      if (seg.size() != 7 || seg[4] != "pods") return status_resp(404, "NotFound", q.path);
      const std::string ns = seg[3], pod = seg[5], verb = seg[6];
      Value in = q.body.empty() ? Value::object() : Value::parse(q.body);
      bool ok = false;
      if (verb == "exec") {
        std::vector<std::string> argv;
        for (auto& a : in.get("command").arr()) argv.push_back(a.str());
        ok = cluster->exec(ns, pod, in.get("container").str(), argv);
      } else if (verb == "kill") {
        Agent* a = cluster->agent_for(ns, pod);
        ok = a && a->kill_pod(ns, pod, (int)in.get("signal").as_int(9));
      } else if (verb == "exit") {
        Agent* a = cluster->agent_for(ns, pod);
        ok = a && a->sim_exit(ns, pod, (int)in.get("code").as_int(0));
      }
      http::Response r;
      r.status = ok ? 200 : 409;
      r.body = ok ? "{\"ok\":true}" : "{\"ok\":false}";
      return r;
    });
  }
}

}  // namespace pdo
