// SPDX-License-Identifier: Apache-2.0
// Minimal HTTP/1.1 server and client (no external dependencies).
//
// Server: one acceptor thread + one thread per connection (the manager, the
// KV server and the local API server serve a handful of clients), keep-alive,
// Content-Length bodies, chunked streaming responses for watches.
// Client: http:// (and https:// when built with OpenSSL, for the Kubernetes
// REST backend), Content-Length and chunked responses, line streaming,
// keep-alive connection reuse; TLS verifies the peer's chain AND host name.
// WebSocket (RFC 6455) both ways: the server upgrades a request
// (Response::upgrade) and ws_exec() speaks the Kubernetes pods/exec
// channel protocol (v5/v4.channel.k8s.io) — the transport the reference's
// start-order coordinator uses (controllers/paddlejob_controller.go:491-518,
// there through SPDY).
// Every socket is close-on-exec: the agent fork+execs ranks from this process.
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace pdo {
namespace http {

struct Request {
  std::string method;
  std::string path;   // without query
  std::string query;  // raw query string
  std::map<std::string, std::string> headers;  // lower-case keys
  std::string body;
  std::string param(const std::string& k, const std::string& def = "") const;
  std::vector<std::string> params(const std::string& k) const;  // repeated keys (?command=a&command=b)
};

class StreamWriter {
 public:
  virtual ~StreamWriter() = default;
  virtual bool write(const std::string& chunk) = 0;  // false → client gone
  virtual bool closed() const = 0;
};

struct Response {
  int status = 200;
  std::string content_type = "application/json";
  std::string body;
  std::map<std::string, std::string> headers;
  // streaming: called after headers are sent (chunked); return when done
  std::function<void(StreamWriter&)> stream;
  // protocol upgrade (status 101): called with the raw connection after the
  // response head; the connection is closed when it returns
  std::function<void(int fd)> upgrade;
};

using Handler = std::function<Response(const Request&)>;

class Server {
 public:
  Server() = default;
  ~Server();
  // exact path or prefix ending in '*'
  void route(const std::string& method, const std::string& path, Handler h);
  // addr ":8080", "127.0.0.1:0", "0" → ephemeral; returns bound port or -1
  int listen(const std::string& addr);
  void start();
  void stop();
  int port() const { return port_; }

 private:
  void accept_loop();
  void serve(int fd);
  const Handler* match(const std::string& method, const std::string& path) const;

  struct Route {
    std::string method, path;
    bool prefix;
    Handler h;
  };
  std::vector<Route> routes_;
  int fd_ = -1;
  int port_ = -1;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex conn_mu_;
  std::vector<int> conn_fds_;
  std::atomic<int> active_{0};
};

struct ClientResponse {
  int status = 0;
  std::string body;
  std::map<std::string, std::string> headers;
  std::string error;  // transport error (status 0)
};

struct ClientOptions {
  double timeout_s = 10;
  std::map<std::string, std::string> headers;
  std::string ca_file, cert_file, key_file;  // TLS (https), PEM files
  std::string ca_pem, cert_pem, key_pem;     // or PEM text (kubeconfig *-data): never written to disk
  bool insecure_skip_verify = false;
  bool keep_alive = true;  // reuse connections to the same server (not for streams)
  // a request whose repetition is harmless: when a reused keep-alive connection
  // returns nothing after the request was written, it is sent again on a fresh
  // connection.  Default: GET / HEAD / OPTIONS only — an empty read does not prove
  // the server never applied a POST / PUT / DELETE (it may have, then reset).
  // A request that could not be written at all is always retried.
  bool idempotent = false;
};

ClientResponse request(const std::string& method, const std::string& url, const std::string& body = "",
                       const ClientOptions& opt = {});
// streaming GET/POST: on_line(line) for every '\n'-terminated line; return false to stop
ClientResponse stream_lines(const std::string& method, const std::string& url, const std::string& body,
                            const std::function<bool(const std::string&)>& on_line, const ClientOptions& opt = {});

bool parse_url(const std::string& url, std::string* scheme, std::string* host, int* port, std::string* path);
std::string url_decode(const std::string& s);
std::string url_encode(const std::string& s);

// ------------------------------------------------------------ WebSocket
enum WsOpcode { kWsText = 1, kWsBinary = 2, kWsClose = 8, kWsPing = 9, kWsPong = 10 };
std::string ws_accept_key(const std::string& client_key);  // base64(SHA-1(key + GUID))
// server side of an upgraded connection (server frames are unmasked)
class WsConn {
 public:
  explicit WsConn(int fd) : fd_(fd) {}
  bool send(int opcode, const std::string& payload);
  // one message (fragments reassembled, pings answered); false on error / timeout / EOF
  bool recv(int* opcode, std::string* payload, double timeout_s);

 private:
  int fd_;
  std::string buf_;
};

struct ExecResult {
  bool ok = false;     // upgraded, a Status arrived, and it says Success
  int exit_code = -1;  // 0 on Success, the ExitCode cause otherwise
  std::string protocol, out, err, status, error;
};
// Kubernetes pods/exec over WebSocket: GET `url` (…/pods/{name}/exec?container=…
// &command=…) with an Upgrade to v5/v4.channel.k8s.io, demultiplex stdout (1) /
// stderr (2), read the channel-3 metav1.Status.  Bounded by opt.timeout_s.
ExecResult ws_exec(const std::string& url, const ClientOptions& opt);

}  // namespace http
}  // namespace pdo
