// SPDX-License-Identifier: Apache-2.0
#include "api.h"

#include <sys/time.h>

#include <cstdio>
#include <ctime>

namespace pdo {
namespace api {

const std::vector<std::string>& role_order() {
  static const std::vector<std::string> order = {kRolePS, kRoleWorker, kRoleHeter};
  return order;
}

std::string training_role(const std::string& role) {
  if (role == kRolePS) return "PSERVER";
  if (role == kRoleWorker) return "TRAINER";
  if (role == kRoleHeter) return "HETER";
  return "";
}

static std::optional<int> opt_int(const Value& v) {
  if (v.is_number()) return (int)v.as_int();
  return std::nullopt;
}

// ----------------------------------------------------------------- ResourceSpec
ResourceSpec ResourceSpec::from_json(const Value& v) {
  ResourceSpec r;
  if (!v.is_object()) return r;
  r.present = true;
  r.replicas = (int)v.get("replicas").as_int(0);
  r.requests = opt_int(v.get("requests"));
  r.limits = opt_int(v.get("limits"));
  r.tmpl = v.get("template");
  return r;
}

Value ResourceSpec::to_json() const {
  Value o = Value::object();
  o["replicas"] = replicas;  // `json:"replicas"` — no omitempty
  if (requests) o["requests"] = *requests;
  if (limits) o["limits"] = *limits;
  // `template` has omitempty on a struct: always serialised by encoding/json
  o["template"] = tmpl.is_null() ? Value::object() : tmpl;
  return o;
}

// ------------------------------------------------------------ SchedulingPolicy
SchedulingPolicy SchedulingPolicy::from_json(const Value& v) {
  SchedulingPolicy s;
  if (!v.is_object()) return s;
  s.present = true;
  s.min_available = opt_int(v.get("minAvailable"));
  s.queue = v.get("queue").str();
  s.priority_class = v.get("priorityClass").str();
  s.min_resources = v.get("minResources");
  return s;
}

Value SchedulingPolicy::to_json() const {
  Value o = Value::object();
  if (min_available) o["minAvailable"] = *min_available;
  if (!queue.empty()) o["queue"] = queue;
  if (!priority_class.empty()) o["priorityClass"] = priority_class;
  if (min_resources.is_object() && min_resources.size()) o["minResources"] = min_resources;
  return o;
}

// ------------------------------------------------------------------------ Spec
const ResourceSpec* Spec::role(const std::string& r) const {
  const ResourceSpec* p = nullptr;
  if (r == kRolePS) p = &ps;
  else if (r == kRoleWorker) p = &worker;
  else if (r == kRoleHeter) p = &heter;
  return (p && p->present) ? p : nullptr;
}
ResourceSpec* Spec::role(const std::string& r) {
  return const_cast<ResourceSpec*>(static_cast<const Spec*>(this)->role(r));
}

Spec Spec::from_json(const Value& v) {
  Spec s;
  s.clean_pod_policy = v.get("cleanPodPolicy").str();
  s.scheduling = SchedulingPolicy::from_json(v.get("schedulingPolicy"));
  s.intranet = v.get("intranet").str();
  s.with_gloo = opt_int(v.get("withGloo"));
  s.ps = ResourceSpec::from_json(v.get("ps"));
  s.worker = ResourceSpec::from_json(v.get("worker"));
  s.heter = ResourceSpec::from_json(v.get("heter"));
  s.elastic = opt_int(v.get("elastic"));
  return s;
}

Value Spec::to_json() const {
  Value o = Value::object();
  if (!clean_pod_policy.empty()) o["cleanPodPolicy"] = clean_pod_policy;
  if (scheduling.present) o["schedulingPolicy"] = scheduling.to_json();
  if (!intranet.empty()) o["intranet"] = intranet;
  if (with_gloo) o["withGloo"] = *with_gloo;
  if (ps.present) o["ps"] = ps.to_json();
  if (worker.present) o["worker"] = worker.to_json();
  if (heter.present) o["heter"] = heter.to_json();
  if (elastic) o["elastic"] = *elastic;
  return o;
}

// -------------------------------------------------------------- ResourceStatus
ResourceStatus ResourceStatus::from_json(const Value& v) {
  ResourceStatus r;
  if (!v.is_object()) return r;
  r.present = true;
  r.pending = (int)v.get("pending").as_int();
  r.starting = (int)v.get("starting").as_int();
  r.running = (int)v.get("running").as_int();
  r.failed = (int)v.get("failed").as_int();
  r.succeeded = (int)v.get("succeeded").as_int();
  r.unknown = (int)v.get("unknown").as_int();
  for (auto& x : v.get("refs").arr()) r.refs.push_back(x);
  return r;
}

Value ResourceStatus::to_json() const {
  Value o = Value::object();
  if (pending) o["pending"] = pending;
  if (starting) o["starting"] = starting;
  if (running) o["running"] = running;
  if (failed) o["failed"] = failed;
  if (succeeded) o["succeeded"] = succeeded;
  if (unknown) o["unknown"] = unknown;
  if (!refs.empty()) {
    Value a = Value::array();
    for (auto& r : refs) a.push_back(r);
    o["refs"] = a;
  }
  return o;
}

// ---------------------------------------------------------------------- Status
const ResourceStatus* Status::role(const std::string& r) const {
  const ResourceStatus* p = nullptr;
  if (r == kRolePS) p = &ps;
  else if (r == kRoleWorker) p = &worker;
  else if (r == kRoleHeter) p = &heter;
  return (p && p->present) ? p : nullptr;
}
ResourceStatus* Status::role(const std::string& r) {
  if (r == kRolePS) return &ps;
  if (r == kRoleWorker) return &worker;
  if (r == kRoleHeter) return &heter;
  return nullptr;
}

Status Status::from_json(const Value& v) {
  Status s;
  s.phase = v.get("phase").str();
  s.mode = v.get("mode").str();
  s.ps = ResourceStatus::from_json(v.get("ps"));
  s.worker = ResourceStatus::from_json(v.get("worker"));
  s.heter = ResourceStatus::from_json(v.get("heter"));
  s.elastic = v.get("elastic").str();
  s.start_time = v.get("startTime").str();
  s.completion_time = v.get("completionTime").str();
  s.observed_generation = v.get("observedGeneration").as_int();
  return s;
}

Value Status::to_json() const {
  Value o = Value::object();
  if (!phase.empty()) o["phase"] = phase;
  if (!mode.empty()) o["mode"] = mode;
  if (ps.present) o["ps"] = ps.to_json();
  if (worker.present) o["worker"] = worker.to_json();
  if (heter.present) o["heter"] = heter.to_json();
  if (!elastic.empty()) o["elastic"] = elastic;
  if (!start_time.empty()) o["startTime"] = start_time;
  if (!completion_time.empty()) o["completionTime"] = completion_time;
  if (observed_generation) o["observedGeneration"] = observed_generation;
  return o;
}

// ------------------------------------------------------------------- PaddleJob
std::string PaddleJob::annotation(const std::string& k) const {
  return metadata.get("annotations").get(k).str();
}
bool PaddleJob::has_annotation(const std::string& k) const { return metadata.get("annotations").has(k); }

std::vector<std::string> PaddleJob::finalizers() const {
  std::vector<std::string> out;
  for (auto& f : metadata.get("finalizers").arr()) out.push_back(f.str());
  return out;
}

PaddleJob PaddleJob::from_json(const Value& v) {
  PaddleJob j;
  j.metadata = v.get("metadata");
  if (!j.metadata.is_object()) j.metadata = Value::object();
  j.spec = Spec::from_json(v.get("spec"));
  j.status = Status::from_json(v.get("status"));
  return j;
}

Value PaddleJob::to_json() const {
  Value o = Value::object();
  o["apiVersion"] = kAPIVersion;
  o["kind"] = kKind;
  o["metadata"] = metadata;
  o["spec"] = spec.to_json();
  o["status"] = status.to_json();
  return o;
}

std::vector<std::string> validate(const PaddleJob& job) {
  std::vector<std::string> errs;
  if (job.name().empty()) errs.push_back("metadata.name is required");
  bool any = false;
  for (auto& r : role_order()) {
    const ResourceSpec* rs = job.spec.role(r);
    if (!rs) continue;
    any = true;
    if (rs->replicas < 0) errs.push_back("spec." + r + ".replicas must be >= 0");
    const Value& cs = rs->tmpl.at_path("spec.containers");
    if (!cs.is_array() || cs.size() == 0)
      errs.push_back("spec." + r + ".template.spec.containers must contain at least one container");
  }
  if (!any) errs.push_back("spec must define at least one of ps / worker / heter");
  if (job.spec.elastic && !job.spec.role(kRoleWorker)) errs.push_back("spec.elastic requires spec.worker");
  // resource names in the reference are <job>-<role>-<idx>; DNS-1123 subdomain ≤ 63 for hostname
  if (job.name().size() > 50) errs.push_back("metadata.name too long for <name>-<role>-<idx> pod hostnames");
  return errs;
}

void set_type_meta(Value& obj, const std::string& api_version, const std::string& kind) {
  if (!obj.has("apiVersion")) obj["apiVersion"] = api_version;
  if (!obj.has("kind")) obj["kind"] = kind;
}

double wall_clock() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

std::string rfc3339(double t) {
  time_t s = (time_t)t;
  struct tm tmv;
  gmtime_r(&s, &tmv);
  char buf[32];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tmv);
  return buf;
}

double parse_rfc3339(const std::string& s) {
  struct tm tmv = {};
  if (!strptime(s.c_str(), "%Y-%m-%dT%H:%M:%S", &tmv)) return 0;
  return (double)timegm(&tmv);
}

}  // namespace api
}  // namespace pdo
