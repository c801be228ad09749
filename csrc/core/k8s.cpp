// SPDX-License-Identifier: Apache-2.0
#include "k8s.h"

#include <unistd.h>

#include <cstdlib>
#include <fstream>
#include <sstream>

#include "apiserver.h"
#include "base64.h"
#include "hostport.h"
#include "kvclient.h"
#include "log.h"
#include "yaml.h"

namespace pdo {
namespace k8s {

using json::Value;

static std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f) return "";
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

bool Config::load(const std::string& kubeconfig, const std::string& master, Config* out, std::string* err) {
  Config c;
  std::string kc = kubeconfig;
  if (kc.empty() && getenv("KUBECONFIG")) kc = getenv("KUBECONFIG");
  const char* host = getenv("KUBERNETES_SERVICE_HOST");
  if (kc.empty() && host) {
    const char* port = getenv("KUBERNETES_SERVICE_PORT");
    const std::string sa = "/var/run/secrets/kubernetes.io/serviceaccount/";
    c.server = std::string("https://") + host + ":" + (port ? port : "443");
    c.token = read_file(sa + "token");
    while (!c.token.empty() && (c.token.back() == '\n' || c.token.back() == ' ')) c.token.pop_back();
    c.ca_file = sa + "ca.crt";
    std::string ns = read_file(sa + "namespace");
    if (!ns.empty()) c.ns = ns;
  } else if (!kc.empty()) {
    std::string text = read_file(kc);
    if (text.empty()) {
      *err = "cannot read kubeconfig " + kc;
      return false;
    }
    Value doc;
    try {
      doc = text.find_first_not_of(" \t\r\n") != std::string::npos && text[text.find_first_not_of(" \t\r\n")] == '{'
                ? Value::parse(text)
                : yaml::parse(text);
    } catch (const std::exception& e) {
      *err = std::string("kubeconfig parse error: ") + e.what();
      return false;
    }
    std::string ctx_name = doc.get("current-context").str();
    Value ctx, cluster, user;
    for (auto& x : doc.get("contexts").arr())
      if (x.get("name").str() == ctx_name || ctx_name.empty()) {
        ctx = x.get("context");
        break;
      }
    for (auto& x : doc.get("clusters").arr())
      if (x.get("name").str() == ctx.get("cluster").str()) cluster = x.get("cluster");
    for (auto& x : doc.get("users").arr())
      if (x.get("name").str() == ctx.get("user").str()) user = x.get("user");
    c.server = cluster.get("server").str();
    c.insecure = cluster.get("insecure-skip-tls-verify").as_bool();
    c.ca_file = cluster.get("certificate-authority").str();
    std::string dec;
    // *-data fields stay in memory (loaded through BIOs by the TLS client)
    if (c.ca_file.empty() && b64decode(cluster.get("certificate-authority-data").str(), &dec) && !dec.empty())
      c.ca_pem = dec;
    c.token = user.get("token").str();
    c.cert_file = user.get("client-certificate").str();
    c.key_file = user.get("client-key").str();
    if (c.cert_file.empty() && b64decode(user.get("client-certificate-data").str(), &dec) && !dec.empty())
      c.cert_pem = dec;
    if (c.key_file.empty() && b64decode(user.get("client-key-data").str(), &dec) && !dec.empty())
      c.key_pem = dec;
    if (!ctx.get("namespace").str().empty()) c.ns = ctx.get("namespace").str();
  }
  if (!master.empty()) c.server = master;
  if (c.server.empty()) {
    *err = "no apiserver: pass --master, --kubeconfig, or run in-cluster";
    return false;
  }
  *out = c;
  return true;
}

http::ClientOptions Config::client(double timeout_s) const {
  http::ClientOptions o;
  o.timeout_s = timeout_s;
  o.ca_file = ca_file;
  o.cert_file = cert_file;
  o.key_file = key_file;
  o.ca_pem = ca_pem;
  o.cert_pem = cert_pem;
  o.key_pem = key_pem;
  o.insecure_skip_verify = insecure;
  if (!token.empty()) o.headers["Authorization"] = "Bearer " + token;
  o.headers["Accept"] = "application/json";
  return o;
}

static const KindInfo& kind_or_throw(const std::string& kind) {
  const KindInfo* k = kind_by_name(kind);
  if (!k) throw std::runtime_error("unknown kind " + kind);
  return *k;
}

Value RestApi::call(const std::string& method, const std::string& path, const std::string& body) {
  auto r = http::request(method, c_.server + path, body, c_.client());
  if (r.status == 0) throw store::ApiError(store::ApiError::Invalid, "apiserver unreachable: " + r.error);
  Value v;
  try {
    v = r.body.empty() ? Value::object() : Value::parse(r.body);
  } catch (const std::exception&) {
    v = Value::object();
  }
  if (r.status >= 200 && r.status < 300) return v;
  const std::string reason = v.get("reason").str();
  const std::string msg = v.get("message").str(r.body);
  if (r.status == 404) throw store::ApiError(store::ApiError::NotFound, msg);
  if (r.status == 409 && reason == "AlreadyExists") throw store::ApiError(store::ApiError::AlreadyExists, msg);
  if (r.status == 409) throw store::ApiError(store::ApiError::Conflict, msg);
  throw store::ApiError(store::ApiError::Invalid, std::to_string(r.status) + " " + msg);
}

Value RestApi::create(const std::string& kind, Value obj) {
  const KindInfo& k = kind_or_throw(kind);
  api::set_type_meta(obj, k.group_version, k.kind);
  return call("POST", collection_path(k, obj.at_path("metadata.namespace").str()), obj.dump());
}

Value RestApi::update(const std::string& kind, Value obj) {
  const KindInfo& k = kind_or_throw(kind);
  api::set_type_meta(obj, k.group_version, k.kind);
  return call("PUT", collection_path(k, obj.at_path("metadata.namespace").str()) + "/" +
                         obj.at_path("metadata.name").str(),
              obj.dump());
}

Value RestApi::update_status(const std::string& kind, Value obj) {
  const KindInfo& k = kind_or_throw(kind);
  api::set_type_meta(obj, k.group_version, k.kind);
  return call("PUT", collection_path(k, obj.at_path("metadata.namespace").str()) + "/" +
                         obj.at_path("metadata.name").str() + "/status",
              obj.dump());
}

void RestApi::remove(const std::string& kind, const std::string& ns, const std::string& name, bool) {
  const KindInfo& k = kind_or_throw(kind);
  call("DELETE", collection_path(k, ns) + "/" + name, "{\"propagationPolicy\":\"Background\"}");
}

Value RestApi::get(const std::string& kind, const std::string& ns, const std::string& name) {
  return call("GET", collection_path(kind_or_throw(kind), ns) + "/" + name, "");
}

Value RestApi::list(const std::string& kind, const std::string& ns, std::string* rv) {
  Value l = call("GET", collection_path(kind_or_throw(kind), ns), "");
  if (rv) *rv = l.at_path("metadata.resourceVersion").str();
  return l;
}

// ------------------------------------------------------------------ informer
void Informer::start() {
  if (running_.exchange(true)) return;
  th_ = std::thread([this] { run(); });
}

void Informer::stop() {
  if (!running_.exchange(false)) return;
  if (th_.joinable()) th_.join();
}

bool apply_watch_event(const std::string& line, store::Store* cache, const std::string& kind, std::string* rv,
                       bool* gone) {
  const KindInfo* k = kind_by_name(kind);
  Value ev;
  try {
    ev = Value::parse(line);
  } catch (const std::exception&) {
    return true;  // a torn or foreign line: skip it, keep the stream
  }
  const std::string type = ev.get("type").str();
  Value obj = ev.get("object");
  if (type == "ERROR") {
    // metav1.Status: 410 Expired / Gone = the resourceVersion was compacted away
    const int code = (int)obj.get("code").as_int();
    *gone = code == 410 || obj.get("reason").str() == "Expired" || obj.get("reason").str() == "Gone";
    return false;
  }
  const std::string orv = obj.at_path("metadata.resourceVersion").str();
  if (!orv.empty()) *rv = orv;
  if (type == "BOOKMARK") return true;  // only the resourceVersion moves
  if (type != "ADDED" && type != "MODIFIED" && type != "DELETED") return true;
  if (k) api::set_type_meta(obj, k->group_version, k->kind);
  if (type == "DELETED")
    cache->mirror_delete(kind, obj.at_path("metadata.namespace").str(), obj.at_path("metadata.name").str());
  else
    cache->mirror_put(kind, obj);
  return true;
}

void Informer::run() {
  const KindInfo* k = kind_by_name(kind_);
  std::string rv;
  bool need_list = true;
  while (running_) {
    if (need_list) {
      try {
        Value l = api_->list(kind_, ns_, &rv);
        std::vector<Value> items;
        for (auto& o : l.get("items").arr()) {
          Value x = o;
          api::set_type_meta(x, k->group_version, k->kind);
          items.push_back(x);
        }
        cache_->mirror_replace(kind_, ns_, items);
        synced_ = true;
        need_list = false;
        ++lists_;
      } catch (const std::exception& e) {
        log::error("informer", "list failed", {{"kind", kind_}, {"error", e.what()}});
        for (int i = 0; i < 20 && running_; ++i) usleep(100000);
        continue;
      }
    }
    // watch from rv until the stream ends: a clean end (server-side timeout)
    // re-watches from the last resourceVersion seen — BOOKMARKs included —
    // an ERROR event or a failed watch request relists (client-go's reflector)
    const std::string url = api_->config().server + collection_path(*k, ns_) +
                            "?watch=true&allowWatchBookmarks=true&timeoutSeconds=" + std::to_string(watch_timeout_s) +
                            "&resourceVersion=" + http::url_encode(rv);
    bool gone = false, ended_by_event = false;
    auto opts = api_->config().client(watch_timeout_s + 30);
    ++watches_;
    auto r = http::stream_lines("GET", url, "", [&](const std::string& line) {
      if (!running_) return false;
      if (!apply_watch_event(line, cache_, kind_, &rv, &gone)) {
        ended_by_event = true;
        return false;
      }
      return true;
    }, opts);
    if (ended_by_event || r.status != 200) {
      need_list = true;
      if (!gone && running_) usleep(200000);  // an unexpected error: back off before relisting
    }
  }
}

// ------------------------------------------------------------------ leader election
bool LeaderElector::try_acquire_or_renew(double now) {
  const std::string ts = api::rfc3339(now);
  Value lease;
  try {
    lease = api_->get("Lease", ns_, name_);
  } catch (const store::ApiError& e) {
    if (e.code != store::ApiError::NotFound) return false;
    Value l = Value::object();
    l["metadata"]["name"] = name_;
    l["metadata"]["namespace"] = ns_;
    l["spec"]["holderIdentity"] = id_;
    l["spec"]["leaseDurationSeconds"] = (int)lease_duration;
    l["spec"]["acquireTime"] = ts;
    l["spec"]["renewTime"] = ts;
    l["spec"]["leaseTransitions"] = 0;
    try {
      api_->create("Lease", l);
      last_renew_ = now;
      return true;
    } catch (const store::ApiError&) {
      return false;
    }
  }
  const std::string holder = lease.at_path("spec.holderIdentity").str();
  const double renew = api::parse_rfc3339(lease.at_path("spec.renewTime").str());
  const double dur = (double)lease.at_path("spec.leaseDurationSeconds").as_int(15);
  if (holder != id_ && !holder.empty() && renew + dur > now) return false;  // someone else holds it
  if (holder != id_) {
    lease["spec"]["holderIdentity"] = id_;
    lease["spec"]["acquireTime"] = ts;
    lease["spec"]["leaseTransitions"] = lease.at_path("spec.leaseTransitions").as_int(0) + 1;
  }
  lease["spec"]["renewTime"] = ts;
  try {
    api_->update("Lease", lease);
    last_renew_ = now;
    return true;
  } catch (const store::ApiError&) {
    return holder == id_ && now - last_renew_ < renew_deadline;
  }
}

// ------------------------------------------------------------------ manager
int run_manager(const std::string& kubeconfig, const std::string& master, const std::string& ns,
                const std::string& mode, bool volcano, const std::string& init_image, const std::string& etcd,
                int port_start, int port_end, bool leader_elect, const std::string& leader_id, int workers,
                std::atomic<bool>* stop, std::atomic<bool>* ready) {
  Config cfg;
  std::string err;
  if (!Config::load(kubeconfig, master, &cfg, &err)) {
    log::error("setup", "unable to load kubeconfig", {{"error", err}});
    return 1;
  }
  RestApi api(cfg);
  store::Store cache;
  std::vector<std::unique_ptr<Informer>> infs;
  std::vector<std::string> kinds = {"PaddleJob", "Pod", "Service", "ConfigMap"};
  if (volcano) kinds.push_back("PodGroup");
  for (auto& k : kinds) infs.emplace_back(new Informer(&api, &cache, k, ns));

  std::unique_ptr<kv::HttpClient> kvc;
  if (!etcd.empty()) kvc.reset(new kv::HttpClient(etcd));
  HostPorts ports(port_start, port_end);
  ControllerOptions co;
  co.plan = mode == "compat" ? plan::Options::compat_defaults() : plan::Options::fast_defaults();
  co.plan.build.init_image = init_image;
  co.plan.volcano = volcano;
  co.plan.kv = kvc != nullptr;
  if (kvc) co.plan.build.etcd_endpoints = kvc->endpoints();
  co.watch_namespace = ns;
  co.workers = workers;
  co.graceful_pod_delete = false;  // the real kubelet handles termination
  // start-order coordinator release (compat / --initImage): `touch goon` in the
  // coord-paddle container through pods/exec over WebSocket, 3 s bound
  // (controllers/paddlejob_controller.go:491-518)
  ExecFn ex = [&cfg](const std::string& pns, const std::string& pod, const std::string& c,
                     const std::vector<std::string>& argv) {
    std::string url = cfg.server + "/api/v1/namespaces/" + http::url_encode(pns) + "/pods/" + http::url_encode(pod) +
                      "/exec?container=" + http::url_encode(c) + "&stdout=true&stderr=true";
    for (auto& a : argv) url += "&command=" + http::url_encode(a);
    http::ClientOptions o = cfg.client(3.0);
    o.headers.erase("Accept");
    const http::ExecResult r = http::ws_exec(url, o);
    if (!r.ok)
      log::error("controller", "exec in pod failed",
                 {{"pod", pns + "/" + pod}, {"container", c}, {"error", r.error},
                  {"exit_code", std::to_string(r.exit_code)}});
    return r.ok;
  };
  Controller ctrl(&cache, &api, kvc.get(), &ports, ex, co);

  char hn[256] = {0};
  gethostname(hn, sizeof hn - 1);
  LeaderElector le(&api, cfg.ns, leader_id, std::string(hn) + "_" + std::to_string(getpid()));
  if (leader_elect) {
    log::info("setup", "attempting to acquire leader lease", {{"lease", cfg.ns + "/" + leader_id}});
    while (!*stop && !le.try_acquire_or_renew(api::wall_clock())) sleep(2);
    if (*stop) return 0;
    log::info("setup", "successfully acquired lease");
  }
  for (auto& i : infs) i->start();
  for (int t = 0; t < 600 && !*stop; ++t) {
    bool all = true;
    for (auto& i : infs) all = all && i->synced();
    if (all) break;
    usleep(100000);
  }
  ctrl.start();
  *ready = true;
  log::info("setup", "starting manager", {{"backend", "k8s"}, {"server", cfg.server}, {"mode", mode}});
  double last_renew = api::wall_clock();
  while (!*stop) {
    for (auto& e : cache.drain()) ctrl.on_event(e);
    cache.wait_events(0.05);
    if (leader_elect && api::wall_clock() - last_renew >= le.retry_period) {
      last_renew = api::wall_clock();
      if (!le.try_acquire_or_renew(last_renew)) {
        log::error("setup", "leader lease lost");
        break;
      }
    }
  }
  ctrl.stop();
  for (auto& i : infs) i->stop();
  return 0;
}

}  // namespace k8s
}  // namespace pdo
