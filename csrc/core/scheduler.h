// SPDX-License-Identifier: Apache-2.0
// Scheduler stand-in for the local backend: default FIFO bin-packing on
// amd.com/gpu + Volcano-style gang admission for PodGroups.
//
// The reference delegates placement to kube-scheduler / Volcano
// (controllers/paddlejob_controller.go:133-157: pods are created only once
// the PodGroup is Inqueue/Running).  Here:
//  * PodGroup Pending → Inqueue when the cluster's free amd.com/gpu (and pod
//    slots) cover minResources / minMember (Volcano's `enqueue` action);
//  * pods with schedulerName=volcano bind only when their group is
//    Inqueue/Running, and a group's first minMember pods bind all-or-nothing
//    (gang); PodGroup → Running once minMember pods run;
//  * every other pod binds FIFO to the first node with enough free GPUs.
#pragma once

#include <map>
#include <set>
#include <string>
#include <vector>

#include "store.h"

namespace pdo {

struct NodeInfo {
  std::string name = "local";
  std::string ip = "127.0.0.1";
  int gpus = 0;             // amd.com/gpu capacity
  int max_pods = 110;
  bool remote = false;  // served by a standalone pdo-agent (no in-process agent)
  std::vector<std::string> gpu_cpulists;  // NUMA-local CPU list per GPU (sysfs local_cpulist)
};

// amd.com/gpu requested by a pod (Σ containers: limits, else requests)
int pod_gpu_request(const json::Value& pod);

class Scheduler {
 public:
  Scheduler(store::Store* s, std::vector<NodeInfo> nodes) : s_(s), nodes_(std::move(nodes)) {}
  // one scheduling pass; returns number of pods bound
  int sync();
  const std::vector<NodeInfo>& nodes() const { return nodes_; }
  std::map<std::string, int> free_gpus() const;

 private:
  bool bind(json::Value pod, const std::string& node);
  store::Store* s_;
  std::vector<NodeInfo> nodes_;
};

}  // namespace pdo
