// SPDX-License-Identifier: Apache-2.0
// Native unit tests of the control plane (no framework dependency).
// Built in the normal build and in sanitizer builds:
//   cmake -DPDO_SANITIZE=address,undefined …   /  -DPDO_SANITIZE=thread …
// (the reference runs no race detector; pdo runs these and the
// multi-worker controller stress below under TSan in CI.)
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "builders.h"
#include "cluster.h"
#include "http.h"
#include "kvclient.h"
#include "kvstore.h"
#include "planner.h"
#include "quantity.h"
#include "store.h"
#include "workqueue.h"
#include "yaml.h"

using pdo::json::Value;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    if (!(cond)) {                                                          \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
      ++g_fail;                                                             \
    } else {                                                                \
      ++g_pass;                                                             \
    }                                                                       \
  } while (0)

static Value job(const std::string& name, int ps, int workers, const std::string& intranet = "") {
  std::string tmpl = R"({"spec":{"containers":[{"name":"c","image":"busybox","command":["sleep","1000"]}]}})";
  Value j = Value::parse(R"({"apiVersion":"batch.paddlepaddle.org/v1","kind":"PaddleJob","metadata":{"name":")" +
                         name + R"(","namespace":"default"},"spec":{}})");
  if (ps) {
    j["spec"]["ps"]["replicas"] = ps;
    j["spec"]["ps"]["template"] = Value::parse(tmpl);
  }
  if (workers) {
    j["spec"]["worker"]["replicas"] = workers;
    j["spec"]["worker"]["template"] = Value::parse(tmpl);
  }
  if (!intranet.empty()) j["spec"]["intranet"] = intranet;
  return j;
}

static void test_json() {
  Value v = Value::parse(R"({"a":[1,2.5,"x",{"b":null}],"c":true,"d":"é\n"})");
  CHECK(v.get("a").size() == 4);
  CHECK(v.get("a")[0].as_int() == 1);
  CHECK(v.get("c").as_bool());
  CHECK(Value::parse(v.dump()) == v);
  CHECK(v.at_path("a").is_array());
  bool threw = false;
  try {
    Value::parse("{\"a\":}");
  } catch (const pdo::json::ParseError&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_quantity() {
  pdo::Quantity a, b;
  CHECK(pdo::Quantity::parse("500m", &a) && pdo::Quantity::parse("500m", &b));
  a.add(b);
  CHECK(a.str() == "1");
  CHECK(pdo::Quantity::parse("2Gi", &a) && pdo::Quantity::parse("2Gi", &b));
  a.add(b);
  CHECK(a.str() == "4Gi");
  CHECK(pdo::Quantity::parse("1000", &a) && a.str() == "1k");
  CHECK(pdo::Quantity::parse("10m", &a) && a.str() == "10m");
}

static void test_builders() {
  auto j = pdo::api::PaddleJob::from_json(job("wd", 2, 2));
  auto nm = pdo::build::extract_name_index("wide-and-deep-worker-12");
  CHECK(nm.first == "worker" && nm.second == 12);
  pdo::build::Options opt;
  Value pod = pdo::build::construct_pod(j, "ps", 1, opt);
  CHECK(pod.at_path("metadata.name").as_string() == "wd-ps-1");
  CHECK(pod.at_path("spec.restartPolicy").as_string() == "Never");
  CHECK(pod.at_path("metadata.labels").get("paddle-res-type").as_string() == "ps");
  const Value& env = pod.at_path("spec.containers")[0].get("env");
  CHECK(env[0].get("name").as_string() == "POD_IP");
  CHECK(env[1].get("value").as_string() == "1");
  CHECK(env[2].get("value").as_string() == "PSERVER");
  std::vector<Value> pods;
  for (int i = 0; i < 2; ++i)
    for (const char* r : {"ps", "worker"}) {
      Value p = pdo::build::construct_pod(j, r, i, opt);
      p["status"]["podIP"] = std::string("10.0.0.") + std::to_string(pods.size() + 1);
      pods.push_back(p);
    }
  Value cm = pdo::build::construct_configmap(j, pods);
  CHECK(cm.at_path("data.PADDLE_TRAINERS_NUM").as_string() == "2");
  CHECK(cm.at_path("data.PADDLE_PSERVERS_IP_PORT_LIST").as_string() == "10.0.0.1:2379,10.0.0.3:2379");
}

static void test_planner_compat_one_mutation() {
  auto j = pdo::api::PaddleJob::from_json(job("x", 0, 3));
  j.metadata["finalizers"] = Value(pdo::json::Array{Value(pdo::api::kFinalizer)});
  pdo::plan::Observed obs;
  obs.job = j;
  auto p = pdo::plan::reconcile(obs, pdo::plan::Options::compat_defaults(), nullptr, 1000);
  int creates = 0;
  for (auto& a : p.actions)
    if (a.op == pdo::plan::Op::CreatePod) ++creates;
  CHECK(creates == 1);
  auto f = pdo::plan::reconcile(obs, pdo::plan::Options::fast_defaults(), nullptr, 1000);
  creates = 0;
  for (auto& a : f.actions)
    if (a.op == pdo::plan::Op::CreatePod) ++creates;
  CHECK(creates == 3);
}

static void test_store_and_gc() {
  pdo::store::Store s;
  Value j = s.create("PaddleJob", job("g", 0, 1));
  Value pod = Value::parse(R"({"metadata":{"name":"g-worker-0","namespace":"default"}})");
  pod["metadata"]["ownerReferences"] = Value(pdo::json::Array{pdo::build::owner_reference(pdo::api::PaddleJob::from_json(j))});
  s.create("Pod", pod);
  CHECK(s.list("Pod", "default", {}, "g").size() == 1);
  bool conflict = false;
  Value stale = j;
  s.update("PaddleJob", j);  // no-op
  Value j2 = j;
  j2["spec"]["worker"]["replicas"] = 2;
  s.update("PaddleJob", j2);
  try {
    stale["spec"]["worker"]["replicas"] = 5;
    s.update("PaddleJob", stale);
  } catch (const pdo::store::ApiError& e) {
    conflict = e.code == pdo::store::ApiError::Conflict;
  }
  CHECK(conflict);
  s.remove("PaddleJob", "default", "g");
  CHECK(s.list("Pod").empty());  // background GC
}

static void test_workqueue() {
  double now = 0;
  pdo::WorkQueue q([&] { return now; });
  q.add("a");
  q.add("a");
  CHECK(q.len() == 1);
  std::string k;
  CHECK(q.get(&k, 0) && k == "a");
  q.add("a");  // while processing
  CHECK(!q.get(&k, 0));
  q.done("a");
  CHECK(q.get(&k, 0) && k == "a");
  q.done("a");
  q.add_after("b", 1.0);
  CHECK(!q.get(&k, 0));
  now = 1.5;
  CHECK(q.get(&k, 0) && k == "b");
  q.done("b");
}

static void test_kv_and_http() {
  pdo::kv::KVStore s;
  std::atomic<int> seen{0};
  s.watch("/paddle/", pdo::kv::KVStore::prefix_end("/paddle/"), 0, [&](int64_t, const std::vector<pdo::kv::Event>& e) {
    seen += (int)e.size();
    return true;
  });
  s.put("/paddle/ns-a/np", "4");
  s.put("/other", "x");
  CHECK(seen == 1);
  pdo::kv::Compare c;
  c.key = "/paddle/ns-a/np";
  c.target = pdo::kv::Compare::Value;
  c.value = "4";
  pdo::kv::Op op;
  op.type = pdo::kv::Op::Put;
  op.key = c.key;
  op.value = "8";
  CHECK(s.txn({c}, {op}, {}, nullptr));
  pdo::kv::KeyValue kv;
  CHECK(s.get("/paddle/ns-a/np", &kv) && kv.value == "8" && kv.version == 2);
  int64_t lease = s.lease_grant(1);
  s.put("/ephemeral", "1", lease);
  CHECK(s.lease_revoke(lease));
  CHECK(!s.get("/ephemeral", nullptr));

  pdo::http::Server srv;
  pdo::kv::mount_gateway(srv, s);
  int port = srv.listen("127.0.0.1:0");
  CHECK(port > 0);
  srv.start();
  pdo::kv::HttpClient cl("127.0.0.1:" + std::to_string(port));
  std::vector<pdo::kv::KeyValue> kvs;
  CHECK(cl.get("/paddle/ns-a/np", &kvs) && kvs.size() == 1 && kvs[0].value == "8");
  CHECK(cl.put("/paddle/ns-a/np", "4"));
  CHECK(s.get("/paddle/ns-a/np", &kv) && kv.value == "4");
  srv.stop();
}

// WebSocket handshake key (RFC 6455 §1.3 example), keep-alive reuse, and a
// pods/exec-style upgrade round trip between the server and ws_exec
static void test_websocket_and_keepalive() {
  CHECK(pdo::http::ws_accept_key("dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=");
  CHECK(pdo::http::url_encode("a b/c&d") == "a%20b%2Fc%26d");
  pdo::http::Server srv;
  std::atomic<int> hits{0};
  srv.route("GET", "/ping", [&](const pdo::http::Request&) {
    ++hits;
    pdo::http::Response r;
    r.body = "{\"ok\":true}";
    return r;
  });
  srv.route("GET", "/exec", [](const pdo::http::Request& q) {
    pdo::http::Response r;
    r.status = 101;
    r.headers["Upgrade"] = "websocket";
    r.headers["Connection"] = "Upgrade";
    r.headers["Sec-WebSocket-Accept"] = pdo::http::ws_accept_key(q.headers.at("sec-websocket-key"));
    r.headers["Sec-WebSocket-Protocol"] = "v4.channel.k8s.io";
    const auto cmd = q.params("command");
    r.upgrade = [cmd](int fd) {
      pdo::http::WsConn ws(fd);
      std::string joined;
      for (auto& c : cmd) joined += c + " ";
      ws.send(pdo::http::kWsBinary, std::string(1, '\x01') + joined);
      ws.send(pdo::http::kWsBinary, std::string(1, '\x02') + std::string(70000, 'e'));  // 64-bit length form
      const std::string ok = "{\"status\":\"Success\"}";
      const std::string bad =
          "{\"status\":\"Failure\",\"message\":\"bad\",\"details\":{\"causes\":[{\"message\":\"7\","
          "\"reason\":\"ExitCode\"}]}}";
      ws.send(pdo::http::kWsBinary, std::string(1, '\x03') + (cmd.size() == 2 ? ok : bad));
      ws.send(pdo::http::kWsClose, "");
    };
    return r;
  });
  int port = srv.listen("127.0.0.1:0");
  CHECK(port > 0);
  srv.start();
  const std::string base = "http://127.0.0.1:" + std::to_string(port);
  for (int i = 0; i < 5; ++i) CHECK(pdo::http::request("GET", base + "/ping").status == 200);
  CHECK(hits == 5);
  auto r = pdo::http::ws_exec(base + "/exec?command=touch&command=goon", {});
  CHECK(r.ok && r.exit_code == 0 && r.out == "touch goon " && r.err.size() == 70000 &&
        r.protocol == "v4.channel.k8s.io");
  auto f = pdo::http::ws_exec(base + "/exec?command=false", {});
  CHECK(!f.ok && f.exit_code == 7 && f.error == "bad");
  auto n = pdo::http::ws_exec(base + "/ping", {});  // no upgrade → refused cleanly
  CHECK(!n.ok && n.error.find("HTTP 200") != std::string::npos);
  srv.stop();
}

static void test_yaml() {
  const char* y = R"(apiVersion: v1
clusters:
- cluster:
    server: https://1.2.3.4:6443   # comment
    insecure-skip-tls-verify: true
  name: c1
users:
- name: u1
  user:
    token: "abc:def"
list: [1, two, "3"]
)";
  Value v = pdo::yaml::parse(y);
  CHECK(v.get("clusters")[0].get("cluster").get("server").as_string() == "https://1.2.3.4:6443");
  CHECK(v.get("clusters")[0].get("cluster").get("insecure-skip-tls-verify").as_bool());
  CHECK(v.get("users")[0].at_path("user.token").as_string() == "abc:def");
  CHECK(v.get("list")[1].as_string() == "two" && v.get("list")[0].as_int() == 1);
}

static void test_cluster_sim_multiworker() {
  pdo::ClusterOptions o;
  o.workers = 4;
  o.agent_mode = pdo::AgentOptions::Sim;
  pdo::Cluster c(o);
  for (int i = 0; i < 8; ++i) c.apply("PaddleJob", job("j" + std::to_string(i), 1, 2));
  c.start();
  for (int t = 0; t < 300; ++t) {
    usleep(10000);
    int running = 0;
    for (auto& j : c.store().list("PaddleJob")) running += j.at_path("status.phase").as_string() == "Running";
    if (running == 8) break;
  }
  int running = 0;
  for (auto& j : c.store().list("PaddleJob")) running += j.at_path("status.phase").as_string() == "Running";
  c.stop();
  CHECK(running == 8);
}

// controller=false: API objects are stored and watched, but nothing reconciles
// them — no pods, no status (the bare cluster an external operator drives)
static void test_cluster_without_controller() {
  pdo::ClusterOptions o;
  o.agent_mode = pdo::AgentOptions::Sim;
  o.controller = false;
  pdo::Cluster c(o);
  c.apply("PaddleJob", job("bare", 1, 2));
  c.start();
  usleep(200000);
  c.stop();
  for (int i = 0; i < 20; ++i) c.tick();
  CHECK(c.store().list("PaddleJob").size() == 1);
  CHECK(c.store().list("Pod").empty());
  CHECK(c.store().list("PaddleJob")[0].at_path("status.phase").as_string().empty());
}

int main() {
  test_json();
  test_quantity();
  test_builders();
  test_planner_compat_one_mutation();
  test_store_and_gc();
  test_workqueue();
  test_kv_and_http();
  test_websocket_and_keepalive();
  test_yaml();
  test_cluster_sim_multiworker();
  test_cluster_without_controller();
  printf("core_tests: %d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
