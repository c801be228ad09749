// SPDX-License-Identifier: Apache-2.0
// Minimal HTTP/1.1 server and client (no external dependencies).
//
// Server: one acceptor thread + one thread per connection (the manager, the
// KV server and the local API server serve a handful of clients), keep-alive,
// Content-Length bodies, chunked streaming responses for watches.
// Client: http:// (and https:// when built with OpenSSL, for the Kubernetes
// REST backend), Content-Length and chunked responses, line streaming.
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
  std::string ca_file, cert_file, key_file;  // TLS (https)
  bool insecure_skip_verify = false;
};

ClientResponse request(const std::string& method, const std::string& url, const std::string& body = "",
                       const ClientOptions& opt = {});
// streaming GET/POST: on_line(line) for every '\n'-terminated line; return false to stop
ClientResponse stream_lines(const std::string& method, const std::string& url, const std::string& body,
                            const std::function<bool(const std::string&)>& on_line, const ClientOptions& opt = {});

bool parse_url(const std::string& url, std::string* scheme, std::string* host, int* port, std::string* path);
std::string url_decode(const std::string& s);

}  // namespace http
}  // namespace pdo
