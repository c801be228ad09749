// SPDX-License-Identifier: Apache-2.0
// Native unit tests of the control plane (no framework dependency).
// Built in the normal build and in sanitizer builds:
//   cmake -DPDO_SANITIZE=address,undefined …   /  -DPDO_SANITIZE=thread …
// (the reference runs no race detector; pdo runs these and the
// multi-worker controller stress below under TSan in CI.)
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "builders.h"
#include "cluster.h"
#include "http.h"
#include "k8s.h"
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

// ---------------------------------------------------------------- raw-socket fixtures
// A scripted TCP server with no pdo HTTP code in it: connection n is handed to
// script(n, fd).  Used to replay hand-built kube-apiserver responses
// (csrc/tests/fixtures/k8s) and to misbehave in ways the pdo server never does.
#ifndef PDO_FIXTURE_DIR
#define PDO_FIXTURE_DIR "csrc/tests/fixtures"
#endif

static std::string fixture(const std::string& rel) {
  FILE* f = fopen((std::string(PDO_FIXTURE_DIR) + "/" + rel).c_str(), "rb");
  if (!f) {
    fprintf(stderr, "missing fixture %s\n", rel.c_str());
    ++g_fail;
    return "";
  }
  std::string s;
  char buf[4096];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  fclose(f);
  while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
  return s;
}

struct RawServer {
  int lfd = -1, port = 0;
  std::thread th;
  std::atomic<bool> stop{false};
  std::vector<std::string> requests;  // request heads in arrival order
  std::mutex mu;
  explicit RawServer(std::function<void(RawServer&, int n, int fd)> script) {
    lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ::bind(lfd, (sockaddr*)&a, sizeof a);
    ::listen(lfd, 16);
    socklen_t len = sizeof a;
    getsockname(lfd, (sockaddr*)&a, &len);
    port = ntohs(a.sin_port);
    th = std::thread([this, script] {
      for (int n = 0; !stop; ++n) {
        pollfd p{lfd, POLLIN, 0};
        if (::poll(&p, 1, 50) != 1) {
          --n;
          continue;
        }
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) break;
        script(*this, n, fd);
        ::close(fd);
      }
    });
  }
  ~RawServer() {
    stop = true;
    th.join();
    ::close(lfd);
  }
  std::string url() const { return "http://127.0.0.1:" + std::to_string(port); }
  // one request (head + Content-Length body); "" when the peer closed
  std::string read_request(int fd) {
    std::string buf;
    char tmp[4096];
    size_t he;
    while ((he = buf.find("\r\n\r\n")) == std::string::npos) {
      ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r <= 0) return "";
      buf.append(tmp, (size_t)r);
    }
    size_t cl = 0, p = buf.find("Content-Length: ");
    if (p != std::string::npos && p < he) cl = (size_t)atol(buf.c_str() + p + 16);
    while (buf.size() < he + 4 + cl) {
      ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r <= 0) break;
      buf.append(tmp, (size_t)r);
    }
    std::lock_guard<std::mutex> g(mu);
    requests.push_back(buf.substr(0, buf.find("\r\n")));
    return buf;
  }
  static void send_all(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
      ssize_t w = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (w <= 0) return;
      off += (size_t)w;
    }
  }
  static void respond(int fd, int code, const std::string& reason, const std::string& body, bool keep) {
    send_all(fd, "HTTP/1.1 " + std::to_string(code) + " " + reason +
                     "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(body.size()) +
                     (keep ? "\r\nConnection: keep-alive" : "\r\nConnection: close") + "\r\n\r\n" + body);
  }
  // a watch response: chunked, one chunk per line (as the apiserver flushes events)
  static void stream(int fd, const std::string& jsonl, bool terminate) {
    send_all(fd, "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n");
    size_t s = 0;
    while (s < jsonl.size()) {
      size_t e = jsonl.find('\n', s);
      if (e == std::string::npos) e = jsonl.size();
      const std::string line = jsonl.substr(s, e - s) + "\n";
      char hex[16];
      snprintf(hex, sizeof hex, "%zx", line.size());
      send_all(fd, std::string(hex) + "\r\n" + line + "\r\n");
      s = e + 1;
    }
    if (terminate) send_all(fd, "0\r\n\r\n");
  }
};

// a reused keep-alive connection whose server reads a POST and then
// closes without replying must NOT replay the POST on a fresh connection (it may
// have been applied); a GET in the same situation is retried.
static void test_keepalive_retry_only_idempotent() {
  std::atomic<int> posts{0}, gets{0};
  RawServer srv([&](RawServer& s, int n, int fd) {
    if (n == 0) {  // GET answered with keep-alive, then the POST read and dropped
      s.read_request(fd);
      RawServer::respond(fd, 200, "OK", "{}", true);
      if (s.read_request(fd).rfind("POST", 0) == 0) ++posts;
      return;  // close without a reply
    }
    if (n == 1) {  // a fresh connection: GET, keep-alive; then a GET read and dropped
      s.read_request(fd);
      RawServer::respond(fd, 200, "OK", "{}", true);
      if (s.read_request(fd).rfind("GET", 0) == 0) ++gets;
      return;
    }
    std::string r = s.read_request(fd);  // the retried GET (or a replayed POST: counted)
    if (r.rfind("POST", 0) == 0) ++posts;
    if (r.rfind("GET", 0) == 0) ++gets;
    RawServer::respond(fd, 200, "OK", "{\"retried\":true}", false);
  });
  pdo::http::ClientOptions o;
  o.timeout_s = 5;
  CHECK(pdo::http::request("GET", srv.url() + "/a", "", o).status == 200);
  auto p = pdo::http::request("POST", srv.url() + "/lease/grant", "{\"TTL\":5}", o);
  CHECK(p.status == 0 && !p.error.empty());  // surfaced to the caller, not replayed
  CHECK(pdo::http::request("GET", srv.url() + "/b", "", o).status == 200);
  auto g = pdo::http::request("GET", srv.url() + "/c", "", o);
  CHECK(g.status == 200 && g.body.find("retried") != std::string::npos);
  CHECK(posts == 1);
  CHECK(gets == 2);
}

// Status bodies of a real apiserver → the controller's ApiError codes
// (AlreadyExists is "create raced, already there", Conflict is "re-read and retry")
static void test_k8s_status_fixtures() {
  const std::string exists = fixture("k8s/status_409_already_exists.json");
  const std::string conflict = fixture("k8s/status_409_conflict.json");
  const std::string notfound = fixture("k8s/status_404_not_found.json");
  const std::string invalid = fixture("k8s/status_422_invalid.json");
  RawServer srv([&](RawServer& s, int, int fd) {
    const std::string r = s.read_request(fd);
    if (r.rfind("POST", 0) == 0 && r.find("paddlejobs") != std::string::npos)
      RawServer::respond(fd, 409, "Conflict", exists, false);
    else if (r.rfind("PUT", 0) == 0 && r.find("/status") != std::string::npos)
      RawServer::respond(fd, 409, "Conflict", conflict, false);
    else if (r.rfind("PUT", 0) == 0)
      RawServer::respond(fd, 422, "Unprocessable Entity", invalid, false);
    else
      RawServer::respond(fd, 404, "Not Found", notfound, false);
  });
  pdo::k8s::Config c;
  c.server = srv.url();
  pdo::k8s::RestApi api(c);
  Value j = job("resnet", 0, 2);
  auto code_of = [](const std::function<void()>& f) {
    try {
      f();
    } catch (const pdo::store::ApiError& e) {
      return (int)e.code;
    }
    return -1;
  };
  CHECK(code_of([&] { api.create("PaddleJob", j); }) == (int)pdo::store::ApiError::AlreadyExists);
  CHECK(code_of([&] { api.update_status("PaddleJob", j); }) == (int)pdo::store::ApiError::Conflict);
  CHECK(code_of([&] { api.update("PaddleJob", j); }) == (int)pdo::store::ApiError::Invalid);
  CHECK(code_of([&] { api.get("Pod", "default", "resnet-worker-7"); }) == (int)pdo::store::ApiError::NotFound);
  // the request paths the apiserver routes on
  std::lock_guard<std::mutex> g(srv.mu);
  CHECK(srv.requests.size() == 4);
  if (srv.requests.size() == 4) {
    CHECK(srv.requests[0] == "POST /apis/batch.paddlepaddle.org/v1/namespaces/default/paddlejobs HTTP/1.1");
    CHECK(srv.requests[1] == "PUT /apis/batch.paddlepaddle.org/v1/namespaces/default/paddlejobs/resnet/status HTTP/1.1");
    CHECK(srv.requests[3] == "GET /api/v1/namespaces/default/pods/resnet-worker-7 HTTP/1.1");
  }
}

// the informer against a scripted LIST / WATCH sequence: a watch that ends
// cleanly resumes from the BOOKMARK's resourceVersion (no relist); an ERROR 410
// Expired event relists; every event lands in the mirrored cache
static void test_k8s_watch_fixtures() {
  const std::string l100 = fixture("k8s/podlist_rv100.json"), l200 = fixture("k8s/podlist_rv200.json");
  const std::string w100 = fixture("k8s/watch_rv100.jsonl"), w150 = fixture("k8s/watch_rv150_expired.jsonl");
  std::atomic<int> lists{0};
  RawServer srv([&](RawServer& s, int, int fd) {
    const std::string r = s.read_request(fd);
    const std::string head = r.substr(0, r.find("\r\n"));
    if (head.find("watch=true") == std::string::npos) {
      RawServer::respond(fd, 200, "OK", lists++ == 0 ? l100 : l200, false);
    } else if (head.find("resourceVersion=100") != std::string::npos) {
      RawServer::stream(fd, w100, true);  // server-side timeout: the stream just ends
    } else if (head.find("resourceVersion=150") != std::string::npos) {
      RawServer::stream(fd, w150, true);
    } else {
      usleep(20000);
      RawServer::stream(fd, "", true);  // quiet watches from rv 200 on
    }
  });
  pdo::k8s::Config c;
  c.server = srv.url();
  pdo::k8s::RestApi api(c);
  pdo::store::Store cache;
  pdo::k8s::Informer inf(&api, &cache, "Pod", "default");
  inf.watch_timeout_s = 5;
  inf.start();
  for (int i = 0; i < 300 && inf.lists() < 2; ++i) usleep(10000);
  for (int i = 0; i < 100 && inf.watches() < 4; ++i) usleep(10000);
  inf.stop();
  std::vector<std::string> reqs;
  {
    std::lock_guard<std::mutex> g(srv.mu);
    reqs = srv.requests;
  }
  CHECK(reqs.size() >= 5);
  if (reqs.size() >= 5) {
    CHECK(reqs[0].find("watch=true") == std::string::npos);
    CHECK(reqs[1].find("watch=true") != std::string::npos && reqs[1].find("resourceVersion=100") != std::string::npos);
    CHECK(reqs[2].find("resourceVersion=150") != std::string::npos);  // resumed from the BOOKMARK
    CHECK(reqs[3].find("watch=true") == std::string::npos);           // 410 Expired → relist
    CHECK(reqs[4].find("resourceVersion=200") != std::string::npos);
  }
  CHECK(inf.lists() == 2);
  // after the relist only worker-0 (with the relisted label) remains; worker-1
  // was ADDED then DELETED by the watches
  auto pods = cache.list("Pod");
  CHECK(pods.size() == 1);
  if (pods.size() == 1) {
    CHECK(pods[0].at_path("metadata.name").str() == "resnet-worker-0");
    CHECK(pods[0].at_path("metadata.labels.relisted").str() == "yes");
    CHECK(pods[0].get("kind").str() == "Pod");
  }
  // the event function on its own: BOOKMARK moves rv only, ERROR 410 ends the stream
  pdo::store::Store c2;
  std::string rv = "100";
  bool gone = false;
  size_t s = 0;
  int applied = 0;
  while (s < w100.size()) {
    size_t e = w100.find('\n', s);
    if (e == std::string::npos) e = w100.size();
    applied += pdo::k8s::apply_watch_event(w100.substr(s, e - s), &c2, "Pod", &rv, &gone);
    s = e + 1;
  }
  CHECK(applied == 3 && rv == "150" && !gone && c2.list("Pod").size() == 2);
  CHECK(!pdo::k8s::apply_watch_event(w150.substr(w150.find('\n') + 1), &c2, "Pod", &rv, &gone) && gone);
  CHECK(pdo::k8s::apply_watch_event("not json", &c2, "Pod", &rv, &gone));  // a torn line is skipped
}

// pods/exec over WebSocket against hand-assembled server frames (RFC 6455
// framing, unmasked; v5.channel.k8s.io): a fragmented stdout message, a ping
// mid-stream (must be answered), a 16-bit-length stderr frame, the channel-3
// Status of a command that exited 3, then a close frame
static void test_k8s_exec_v5_fixture() {
  const std::string status = fixture("k8s/exec_status_exit3.json");
  std::atomic<bool> got_pong{false};
  RawServer srv([&](RawServer& s, int, int fd) {
    const std::string r = s.read_request(fd);
    size_t k = r.find("Sec-WebSocket-Key: ");
    const std::string key = r.substr(k + 19, r.find("\r\n", k) - k - 19);
    RawServer::send_all(fd, "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                            "Sec-WebSocket-Accept: " + pdo::http::ws_accept_key(key) +
                                "\r\nSec-WebSocket-Protocol: v5.channel.k8s.io\r\n\r\n");
    auto frame = [](unsigned char b0, const std::string& payload) {
      std::string f(1, (char)b0);
      if (payload.size() < 126) {
        f.push_back((char)payload.size());
      } else {
        f.push_back((char)126);
        f.push_back((char)(payload.size() >> 8));
        f.push_back((char)(payload.size() & 0xff));
      }
      return f + payload;
    };
    RawServer::send_all(fd, frame(0x82, std::string(1, '\x01')));          // stream init (channel byte only)
    RawServer::send_all(fd, frame(0x02, std::string("\x01") + "hel"));      // binary, FIN = 0
    RawServer::send_all(fd, frame(0x89, "hb"));                             // ping between fragments
    // the client answers the ping as soon as it reads it: take its pong (masked,
    // opcode 0xA) here, while the stream is still open (reading it only after the
    // close let the client's close race the read)
    char buf[512];
    size_t have = 0;
    for (int tries = 0; have < 2 && tries < 200; ++tries) {
      const ssize_t n = ::recv(fd, buf + have, sizeof buf - have, 0);
      if (n <= 0) break;
      have += (size_t)n;
    }
    if (have >= 2 && ((unsigned char)buf[0] & 0x0f) == 0x0a) got_pong = true;
    RawServer::send_all(fd, frame(0x80, "lo\n"));                           // continuation, FIN = 1
    RawServer::send_all(fd, frame(0x82, std::string("\x02") + std::string(300, 'e')));
    RawServer::send_all(fd, frame(0x82, std::string("\x03") + status));
    RawServer::send_all(fd, frame(0x88, std::string("\x03\xe8", 2)));      // close 1000
    usleep(20000);
  });
  pdo::http::ClientOptions o;
  o.timeout_s = 5;
  auto r = pdo::http::ws_exec(srv.url() + "/api/v1/namespaces/default/pods/p/exec?container=c&command=sh", o);
  CHECK(r.protocol == "v5.channel.k8s.io");
  CHECK(r.out == "hello\n");
  CHECK(r.err == std::string(300, 'e'));
  CHECK(!r.ok && r.exit_code == 3);
  CHECK(r.error.find("exit code 3") != std::string::npos);
  CHECK(got_pong);
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
  test_keepalive_retry_only_idempotent();
  test_k8s_status_fixtures();
  test_k8s_watch_fixtures();
  test_k8s_exec_v5_fixture();
  test_yaml();
  test_cluster_sim_multiworker();
  test_cluster_without_controller();
  printf("core_tests: %d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
