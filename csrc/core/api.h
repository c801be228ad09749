// SPDX-License-Identifier: Apache-2.0
// PaddleJob API (batch.paddlepaddle.org/v1) for the pdo control plane.
//
// Schema parity with the reference CRD (api/v1/paddlejob_types.go:25-281):
// same group/version/kind, field names, omitempty behaviour and enum strings.
// User PodTemplates stay JSON (round-tripped untouched except for the fields
// the builders mutate).  See SURVEY.md Appendix E for the field table.
#pragma once

#include <functional>
#include <optional>
#include <string>
#include <vector>

#include "json.h"

namespace pdo {
namespace api {

using json::Value;

// ---- identity (api/v1/groupversion_info.go:25-34, paddlejob_types.go:218-232)
inline constexpr const char* kGroup = "batch.paddlepaddle.org";
inline constexpr const char* kVersion = "v1";
inline constexpr const char* kAPIVersion = "batch.paddlepaddle.org/v1";
inline constexpr const char* kKind = "PaddleJob";
inline constexpr const char* kListKind = "PaddleJobList";
inline constexpr const char* kPlural = "paddlejobs";
inline constexpr const char* kShortName = "pdj";

// ---- labels / annotations (paddlejob_types.go:29-35)
inline constexpr const char* kLabelResourceName = "paddle-res-name";
inline constexpr const char* kLabelResourceType = "paddle-res-type";
inline constexpr const char* kAnnotationResource = "paddle-resource";
inline constexpr const char* kAnnotationHostPort = "host-port";
// native start-order barrier (fast mode, local backend): "hold" until the
// controller flips it to "released" in ps → worker → heter order; the
// kubelet-lite agent does not start a held pod's main containers.  Replaces
// the busybox init container + `kubectl exec touch goon` of the reference
// (paddlejob_controller.go:308-330,491-518) with one event-driven API write.
inline constexpr const char* kAnnotationStartGate = "pdo.amd.com/start-gate";
inline constexpr const char* kGateHold = "hold";
inline constexpr const char* kGateReleased = "released";
inline constexpr const char* kFinalizer = "finalizers.paddlepaddle.org";

// ---- roles (paddlejob_types.go:37-48) in start order ps → worker → heter
inline constexpr const char* kRolePS = "ps";
inline constexpr const char* kRoleWorker = "worker";
inline constexpr const char* kRoleHeter = "heter";
const std::vector<std::string>& role_order();
std::string training_role(const std::string& role);  // PSERVER / TRAINER / HETER

// ---- ports (controllers/paddlejob_controller.go:49-55)
inline constexpr int kPaddlePort = 2379;
inline constexpr int kPortsPerPod = 20;

// ---- enums (paddlejob_types.go:50-110) — kept as strings like the CRD
namespace phase {
inline constexpr const char* Starting = "Starting";
inline constexpr const char* Pending = "Pending";
inline constexpr const char* Scaling = "Scaling";
inline constexpr const char* Aborting = "Aborting";
inline constexpr const char* Aborted = "Aborted";
inline constexpr const char* Running = "Running";
inline constexpr const char* Restarting = "Restarting";
inline constexpr const char* Completing = "Completing";
inline constexpr const char* Completed = "Completed";
inline constexpr const char* Terminating = "Terminating";
inline constexpr const char* Terminated = "Terminated";
inline constexpr const char* Failed = "Failed";
inline constexpr const char* Succeed = "Succeed";
inline constexpr const char* Unknown = "Unknown";
}  // namespace phase
namespace mode {
inline constexpr const char* PS = "PS";
inline constexpr const char* Collective = "Collective";
inline constexpr const char* Single = "Single";
}  // namespace mode
namespace clean {
inline constexpr const char* Always = "Always";
inline constexpr const char* Never = "Never";
inline constexpr const char* OnFailure = "OnFailure";
inline constexpr const char* OnCompletion = "OnCompletion";
}  // namespace clean
namespace intranet {
inline constexpr const char* PodIP = "PodIP";
inline constexpr const char* Service = "Service";
inline constexpr const char* Host = "Host";
}  // namespace intranet
namespace elastic_status {
inline constexpr const char* None = "NONE";
inline constexpr const char* Doing = "DOING";
inline constexpr const char* Done = "DONE";
inline constexpr const char* Error = "ERROR";
}  // namespace elastic_status

struct ResourceSpec {
  bool present = false;
  int replicas = 0;
  std::optional<int> requests;  // elastic min (declared, never read by the reference)
  std::optional<int> limits;    // elastic max
  Value tmpl;                   // corev1.PodTemplateSpec as JSON
  static ResourceSpec from_json(const Value& v);
  Value to_json() const;
};

struct SchedulingPolicy {
  bool present = false;
  std::optional<int> min_available;
  std::string queue;
  std::string priority_class;
  Value min_resources;  // ResourceList (object) or null
  static SchedulingPolicy from_json(const Value& v);
  Value to_json() const;
};

struct Spec {
  std::string clean_pod_policy;
  SchedulingPolicy scheduling;
  std::string intranet;
  std::optional<int> with_gloo;
  ResourceSpec ps, worker, heter;
  std::optional<int> elastic;

  const ResourceSpec* role(const std::string& r) const;  // nullptr if absent
  ResourceSpec* role(const std::string& r);
  static Spec from_json(const Value& v);
  Value to_json() const;
};

struct ResourceStatus {
  bool present = false;
  int pending = 0, starting = 0, running = 0, failed = 0, succeeded = 0, unknown = 0;
  std::vector<Value> refs;  // corev1.ObjectReference
  static ResourceStatus from_json(const Value& v);
  Value to_json() const;  // omitempty on every field
};

struct Status {
  std::string phase;
  std::string mode;
  ResourceStatus ps, worker, heter;
  std::string elastic;  // ElasticStatus (never set by the reference)
  std::string start_time;
  std::string completion_time;
  int64_t observed_generation = 0;

  const ResourceStatus* role(const std::string& r) const;
  ResourceStatus* role(const std::string& r);
  static Status from_json(const Value& v);
  Value to_json() const;
};

struct PaddleJob {
  Value metadata;  // ObjectMeta as JSON
  Spec spec;
  Status status;

  const std::string& name() const { return metadata.get("name").as_string(); }
  const std::string& ns() const { return metadata.get("namespace").as_string(); }
  const std::string& uid() const { return metadata.get("uid").as_string(); }
  std::string annotation(const std::string& k) const;
  bool has_annotation(const std::string& k) const;
  bool deleting() const { return !metadata.get("deletionTimestamp").is_null(); }
  std::vector<std::string> finalizers() const;
  int64_t generation() const { return metadata.get("generation").as_int(0); }

  static PaddleJob from_json(const Value& v);
  Value to_json() const;
};

// validation errors (empty = valid); permissive like the reference CRD except
// for shapes that would crash the builders (no container in a role template)
std::vector<std::string> validate(const PaddleJob& job);

// apply defaults the apiserver would (kind/apiVersion); no semantic defaults
void set_type_meta(Value& obj, const std::string& api_version, const std::string& kind);

// ---- clock (injectable for deterministic tests) ----------------------------
using Clock = std::function<double()>;  // seconds since epoch
double wall_clock();
std::string rfc3339(double t);  // metav1.Time wire format (second precision, UTC)
double parse_rfc3339(const std::string& s);

}  // namespace api
}  // namespace pdo
