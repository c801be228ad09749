// SPDX-License-Identifier: Apache-2.0
// Kubernetes-compatible REST front end over store::Store (local backend).
//
// Same paths, verbs and list/watch wire format as kube-apiserver for the
// kinds the operator touches, so `pdoctl`, the Python client — and kubectl
// pointed at --server=http://<manager> — work unchanged against the local
// backend:
//   /api/v1/namespaces/{ns}/{pods|services|configmaps|events}[/{name}[/status]]
//   /api/v1/{pods|services|configmaps|events}                (all namespaces)
//   /apis/batch.paddlepaddle.org/v1/namespaces/{ns}/paddlejobs[/{name}[/status]]
//   /apis/batch.paddlepaddle.org/v1/paddlejobs
//   /apis/scheduling.volcano.sh/v1beta1/namespaces/{ns}/podgroups[/{name}]
//   /apis/coordination.k8s.io/v1/namespaces/{ns}/leases[/{name}]
//   ?watch=true streams {"type":"ADDED|MODIFIED|DELETED","object":{…}} lines
//   ?labelSelector=a=b,c=d
//   GET|POST /api/v1/namespaces/{ns}/pods/{name}/exec?container=c&command=…  (WebSocket,
//     v5/v4.channel.k8s.io — what the k8s backend's coordinator and kubectl use)
// plus local-backend extras (no kubelet API exists here):
//   POST /pdo/v1/namespaces/{ns}/pods/{name}/exec   {"container": "...", "command": [...]}
//   POST /pdo/v1/namespaces/{ns}/pods/{name}/kill   {"signal": 9}
#pragma once

#include <functional>
#include <string>
#include <vector>

#include "http.h"
#include "store.h"

namespace pdo {

class Cluster;

struct KindInfo {
  std::string kind, group_version, plural;
  bool namespaced = true;
};

const std::vector<KindInfo>& known_kinds();
const KindInfo* kind_by_plural(const std::string& plural);
const KindInfo* kind_by_name(const std::string& kind);
// REST collection path for a kind in a namespace
std::string collection_path(const KindInfo& k, const std::string& ns);

// fans store watch events out to HTTP watchers (call publish() from the loop)
class WatchHub {
 public:
  int subscribe(std::function<bool(const store::WatchEvent&)> fn);
  void unsubscribe(int id);
  void publish(const store::WatchEvent& ev);

 private:
  std::mutex mu_;
  std::map<int, std::function<bool(const store::WatchEvent&)>> subs_;
  int next_ = 1;
};

void mount_apiserver(http::Server& srv, store::Store& st, WatchHub& hub, Cluster* cluster);

}  // namespace pdo
