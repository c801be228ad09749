// SPDX-License-Identifier: Apache-2.0
// pdo-kv: standalone etcd-v3-subset server (JSON gateway API).
// Replaces deploy/elastic/etcd.yaml's bitnami/etcd for elastic PaddleJobs and
// the launcher rendezvous.  Usage:
//   pdo-kv [--listen-client-urls http://0.0.0.0:2379] [--data-dir DIR]
// --data-dir persists a snapshot on SIGTERM and every --snapshot-interval s.
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

#include "base64.h"
#include "http.h"
#include "json.h"
#include "kvclient.h"
#include "kvstore.h"
#include "log.h"
#include "metrics.h"

static std::atomic<bool> g_stop{false};
static void on_sig(int) { g_stop = true; }

static std::string strip_scheme(std::string u) {
  size_t p = u.find("://");
  if (p != std::string::npos) u = u.substr(p + 3);
  size_t c = u.find(',');
  if (c != std::string::npos) u = u.substr(0, c);
  return u;
}

static void save(pdo::kv::KVStore& s, const std::string& dir) {
  if (dir.empty()) return;
  pdo::json::Value snap = pdo::json::Value::object();
  snap["revision"] = s.revision();
  pdo::json::Value kvs = pdo::json::Value::array();
  for (auto& kv : s.range(std::string(1, '\0'), std::string(1, '\0'))) {
    if (kv.lease) continue;  // leased keys die with their session
    pdo::json::Value o = pdo::json::Value::object();
    o["k"] = pdo::b64encode(kv.key);
    o["v"] = pdo::b64encode(kv.value);
    kvs.push_back(o);
  }
  snap["kvs"] = kvs;
  const std::string tmp = dir + "/snapshot.json.tmp";
  std::ofstream f(tmp);
  f << snap.dump();
  f.close();
  rename(tmp.c_str(), (dir + "/snapshot.json").c_str());
}

static void load(pdo::kv::KVStore& s, const std::string& dir) {
  if (dir.empty()) return;
  std::ifstream f(dir + "/snapshot.json");
  if (!f) return;
  std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  try {
    auto snap = pdo::json::Value::parse(text);
    for (auto& o : snap.get("kvs").arr()) {
      std::string k, v;
      pdo::b64decode(o.get("k").str(), &k);
      pdo::b64decode(o.get("v").str(), &v);
      s.put(k, v);
    }
  } catch (const std::exception& e) {
    pdo::log::error("pdo-kv", "snapshot load failed", {{"error", e.what()}});
  }
}

int main(int argc, char** argv) {
  std::string listen = "0.0.0.0:2379", data_dir;
  double snap_every = 30;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const std::string& flag) -> std::string {
      if (a.rfind(flag + "=", 0) == 0) return a.substr(flag.size() + 1);
      if (a == flag && i + 1 < argc) return argv[++i];
      return "";
    };
    std::string v;
    if (!(v = val("--listen-client-urls")).empty()) listen = strip_scheme(v);
    else if (!(v = val("--data-dir")).empty()) data_dir = v;
    else if (!(v = val("--snapshot-interval")).empty()) snap_every = atof(v.c_str());
    else if (a == "-h" || a == "--help") {
      printf("pdo-kv [--listen-client-urls http://0.0.0.0:2379] [--data-dir DIR] [--snapshot-interval S]\n");
      return 0;
    }
  }
  signal(SIGTERM, on_sig);
  signal(SIGINT, on_sig);
  pdo::kv::KVStore store;
  load(store, data_dir);
  pdo::http::Server srv;
  pdo::kv::mount_gateway(srv, store);
  srv.route("GET", "/metrics", [](const pdo::http::Request&) {
    pdo::http::Response r;
    r.content_type = "text/plain; version=0.0.4";
    r.body = pdo::Metrics::global().expose();
    return r;
  });
  int port = srv.listen(listen);
  if (port < 0) {
    fprintf(stderr, "pdo-kv: cannot listen on %s\n", listen.c_str());
    return 1;
  }
  srv.start();
  pdo::log::info("pdo-kv", "serving", {{"address", listen}, {"port", std::to_string(port)}});
  double since = 0;
  while (!g_stop) {
    usleep(100000);
    store.expire_leases();
    since += 0.1;
    if (since >= snap_every) {
      save(store, data_dir);
      since = 0;
    }
  }
  save(store, data_dir);
  srv.stop();
  return 0;
}
