// SPDX-License-Identifier: Apache-2.0
// Pure object builders: PaddleJob → Pod / ConfigMap / Service / PodGroup.
//
// Behavioural parity with controllers/paddlejob_helper.go (constructPod
// :281-377, constructConfigMap :215-279, constructService4Pod :432-455,
// constructPodGroup/getPGMinResource :478-549, naming :201-213/:396-403) plus
// the create-time additions of the reconciler (coordinator init container,
// Volcano annotations, elastic etcd endpoint: paddlejob_controller.go:234-275).
//
// MI355X-first additions (documented deviations, all opt-out via options):
//  * gpu_resource_rewrite: `nvidia.com/gpu` requests/limits in user templates
//    are rewritten to `amd.com/gpu` so reference manifests schedule on MI355X
//    nodes (no NVIDIA device-plugin path exists in this framework);
//  * rank env for the PyTorch-ROCm launcher (PDO_JOB / PDO_ROLE /
//    PDO_REPLICA_INDEX / PDO_REPLICAS) next to the Paddle contract;
//  * every env var / port is added to EVERY container that lacks it is NOT
//    done: like the reference only Containers[0] is mutated (quirk D-11).
#pragma once

#include <string>
#include <utility>
#include <vector>

#include "api.h"

namespace pdo {
namespace build {

using json::Value;

inline constexpr const char* kCoordContainer = "coord-paddle";
inline constexpr const char* kSchedulerVolcano = "volcano";
inline constexpr const char* kPodGroupAnnotation = "scheduling.k8s.io/group-name";
inline constexpr const char* kVolcanoTaskSpec = "volcano.sh/task-spec";
inline constexpr const char* kVolcanoJobName = "volcano.sh/job-name";
inline constexpr const char* kVolcanoJobVersion = "volcano.sh/job-version";
inline constexpr const char* kVolcanoQueueName = "volcano.sh/queue-name";
inline constexpr const char* kAMDGPU = "amd.com/gpu";
inline constexpr const char* kNVGPU = "nvidia.com/gpu";

struct Options {
  std::string init_image;                   // "" disables the coordinator
  bool volcano = false;                     // --scheduling=volcano
  std::vector<std::string> etcd_endpoints;  // --etcd-server (elastic)
  bool gpu_resource_rewrite = true;
  bool launcher_env = true;
  // native start-order barrier (kAnnotationStartGate): pods of every role after
  // the first one present are created held; no effect with an init image
  bool start_gate = false;
};

// true if pods of `role` are created held by the native start gate
bool start_gated(const api::PaddleJob& job, const std::string& role, const Options& opt);

std::string res_name(const std::string& job, const std::string& role, int idx);
// "<job>-<role>-<idx>" → (role, idx); ("", 0) when the tail is not an int
std::pair<std::string, int> extract_name_index(const std::string& name);
std::string endpoints_to_hosts(const std::vector<std::string>& eps);
std::string gen_endpoints(const std::string& job, const std::string& role, int n, int port);

Value owner_reference(const api::PaddleJob& job);
void set_controller_reference(Value& obj, const api::PaddleJob& job);
// controller owner name if the controller is a PaddleJob (the field index)
std::string controller_owner(const Value& obj);
Value object_reference(const Value& obj, const std::string& api_version, const std::string& kind);

Value coord_init_container(const std::string& image);
bool without_volcano(const api::PaddleJob& job);

// full pod as the reconciler creates it (constructPod + createPod additions)
Value construct_pod(const api::PaddleJob& job, const std::string& role, int idx, const Options& opt);
// nullptr-equivalent (Null value) when some pod has no IPv4 yet.
// host_port_endpoints: Host-mode endpoints carry the job's allocated host port
// (fast mode) instead of the reference's fixed :2379 (SURVEY D-5, compat mode)
Value construct_configmap(const api::PaddleJob& job, const std::vector<Value>& pods,
                          bool host_port_endpoints = false);
Value construct_service_for_pod(const Value& pod);
Value construct_podgroup(const api::PaddleJob& job, bool rewrite_gpu = true);
Value pg_min_resources(const api::PaddleJob& job, bool rewrite_gpu = true);
int total_replicas(const api::PaddleJob& job);

}  // namespace build
}  // namespace pdo
