// SPDX-License-Identifier: Apache-2.0
// etcd-v3 JSON-gateway front end for KVStore + a matching client.
//
// Routes (POST, JSON bodies, base64 keys/values, int64 as strings — the
// grpc-gateway conventions of etcd ≥ 3.4):
//   /v3/kv/range  /v3/kv/put  /v3/kv/deleterange  /v3/kv/txn
//   /v3/lease/grant  /v3/lease/revoke  /v3/lease/keepalive  /v3/lease/timetolive
//   /v3/watch     (streaming: one JSON object per line)
//   GET /health   GET /metrics
// The controller's elastic `np` sync (reference controllers/paddlejob_elastic.go)
// and the launcher's rendezvous talk to pdo-kv or to a real etcd through
// this one API.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "http.h"
#include "kvstore.h"

namespace pdo {
namespace kv {

void mount_gateway(http::Server& srv, KVStore& store);

// abstract KV access used by the controller (in-process store or remote)
class Client {
 public:
  virtual ~Client() = default;
  // returns false on transport error; *kvs gets all kvs under `key` (exact)
  virtual bool get(const std::string& key, std::vector<KeyValue>* kvs) = 0;
  virtual bool put(const std::string& key, const std::string& value) = 0;
  virtual std::vector<std::string> endpoints() const = 0;
};

class LocalClient : public Client {
 public:
  explicit LocalClient(KVStore* s, std::string ep = "inproc://pdo-kv") : s_(s), ep_(std::move(ep)) {}
  bool get(const std::string& key, std::vector<KeyValue>* kvs) override;
  bool put(const std::string& key, const std::string& value) override;
  std::vector<std::string> endpoints() const override { return {ep_}; }

 private:
  KVStore* s_;
  std::string ep_;
};

class HttpClient : public Client {
 public:
  // endpoints "host:port,host2:port" (etcd --etcd-server syntax); 3 s op timeout (paddlejob_elastic.go:42)
  explicit HttpClient(const std::string& endpoints, double timeout_s = 3.0);
  bool get(const std::string& key, std::vector<KeyValue>* kvs) override;
  bool put(const std::string& key, const std::string& value) override;
  std::vector<std::string> endpoints() const override { return eps_; }

 private:
  bool call(const std::string& path, const std::string& body, std::string* out);
  std::vector<std::string> eps_;
  double timeout_;
};

}  // namespace kv
}  // namespace pdo
