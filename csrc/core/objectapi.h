// SPDX-License-Identifier: Apache-2.0
// Write side of the API used by the controller and the agent: the local
// store (StoreApi) or a remote apiserver (k8s::RestApi).
#pragma once

#include <string>

#include "store.h"

namespace pdo {

class ObjectApi {
 public:
  virtual ~ObjectApi() = default;
  virtual json::Value create(const std::string& kind, json::Value obj) = 0;
  virtual json::Value update(const std::string& kind, json::Value obj) = 0;
  virtual json::Value update_status(const std::string& kind, json::Value obj) = 0;
  // graceful: let the kubelet terminate the pod (deletionTimestamp first)
  virtual void remove(const std::string& kind, const std::string& ns, const std::string& name, bool graceful) = 0;
};

class StoreApi : public ObjectApi {
 public:
  explicit StoreApi(store::Store* s) : s_(s) {}
  json::Value create(const std::string& kind, json::Value obj) override { return s_->create(kind, std::move(obj)); }
  json::Value update(const std::string& kind, json::Value obj) override { return s_->update(kind, std::move(obj)); }
  json::Value update_status(const std::string& kind, json::Value obj) override {
    return s_->update_status(kind, std::move(obj));
  }
  void remove(const std::string& kind, const std::string& ns, const std::string& name, bool graceful) override {
    s_->remove(kind, ns, name, graceful);
  }

 private:
  store::Store* s_;
};

}  // namespace pdo
