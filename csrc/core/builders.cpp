// SPDX-License-Identifier: Apache-2.0
#include "builders.h"

#include <cstdlib>
#include <map>

#include "quantity.h"

namespace pdo {
namespace build {

using api::PaddleJob;

std::string res_name(const std::string& job, const std::string& role, int idx) {
  return job + "-" + role + "-" + std::to_string(idx);
}

std::pair<std::string, int> extract_name_index(const std::string& name) {
  size_t last = name.rfind('-');
  if (last == std::string::npos) return {"", 0};
  std::string tail = name.substr(last + 1);
  if (tail.empty()) return {"", 0};
  char* end = nullptr;
  long v = strtol(tail.c_str(), &end, 10);
  if (!end || *end) return {"", 0};
  size_t prev = name.rfind('-', last - 1);
  std::string role = prev == std::string::npos ? name.substr(0, last) : name.substr(prev + 1, last - prev - 1);
  if (last == 0) role = "";
  return {role, (int)v};
}

std::string endpoints_to_hosts(const std::vector<std::string>& eps) {
  std::string out;
  for (size_t i = 0; i < eps.size(); ++i) {
    if (i) out += ",";
    out += eps[i].substr(0, eps[i].find(':'));
  }
  return out;
}

std::string gen_endpoints(const std::string& job, const std::string& role, int n, int port) {
  std::string out;
  for (int i = 0; i < n; ++i) {
    if (i) out += ",";
    out += res_name(job, role, i) + ":" + std::to_string(port);
  }
  return out;
}

static std::string join(const std::vector<std::string>& v, const char* sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

Value owner_reference(const PaddleJob& job) {
  Value r = Value::object();
  r["apiVersion"] = api::kAPIVersion;
  r["kind"] = api::kKind;
  r["name"] = job.name();
  r["uid"] = job.uid();
  r["controller"] = true;
  r["blockOwnerDeletion"] = true;
  return r;
}

void set_controller_reference(Value& obj, const PaddleJob& job) {
  Value& refs = obj["metadata"]["ownerReferences"];
  if (!refs.is_array()) refs = Value::array();
  for (auto& r : refs.arr())
    if (r.get("controller").as_bool()) return;  // already controlled
  refs.push_back(owner_reference(job));
}

std::string controller_owner(const Value& obj) {
  for (auto& r : obj.at_path("metadata.ownerReferences").arr()) {
    if (!r.get("controller").as_bool()) continue;
    if (r.get("apiVersion").as_string() != api::kAPIVersion || r.get("kind").as_string() != api::kKind) return "";
    return r.get("name").str();
  }
  return "";
}

Value object_reference(const Value& obj, const std::string& api_version, const std::string& kind) {
  Value r = Value::object();
  r["kind"] = kind;
  const Value& md = obj.get("metadata");
  if (!md.get("namespace").as_string().empty()) r["namespace"] = md.get("namespace");
  r["name"] = md.get("name");
  if (!md.get("uid").as_string().empty()) r["uid"] = md.get("uid");
  r["apiVersion"] = api_version;
  if (!md.get("resourceVersion").as_string().empty()) r["resourceVersion"] = md.get("resourceVersion");
  return r;
}

Value coord_init_container(const std::string& image) {
  Value c = Value::object();
  c["name"] = kCoordContainer;
  c["image"] = image;
  c["command"] = Value(json::Array{Value("sh"), Value("-c"),
                                   Value("while true; do if [ -f goon ]; then exit 0; else sleep 0.1; fi; done")});
  Value req = Value::object();
  req["cpu"] = "10m";
  req["memory"] = "10m";
  c["resources"]["requests"] = req;
  c["imagePullPolicy"] = "IfNotPresent";
  return c;
}

bool without_volcano(const PaddleJob& job) {
  for (auto& r : api::role_order()) {
    const api::ResourceSpec* rs = job.spec.role(r);
    if (!rs) continue;
    const std::string& s = rs->tmpl.at_path("spec.schedulerName").as_string();
    if (!s.empty() && s != kSchedulerVolcano) return true;
  }
  return false;
}

static Value env(const std::string& name, const std::string& value) {
  Value e = Value::object();
  e["name"] = name;
  e["value"] = value;
  return e;
}

static void rewrite_gpu_resources(Value& container) {
  for (const char* kind : {"requests", "limits"}) {
    Value* rl = container["resources"].find(kind);
    if (!rl || !rl->is_object()) continue;
    Value* nv = rl->find(kNVGPU);
    if (!nv) continue;
    Value q = *nv;
    rl->erase(kNVGPU);
    if (!rl->has(kAMDGPU)) (*rl)[kAMDGPU] = q;
  }
  if (container["resources"].size() == 0) container.erase("resources");
}

bool start_gated(const PaddleJob& job, const std::string& role, const Options& opt) {
  if (!opt.start_gate || !opt.init_image.empty()) return false;
  // ordering only matters between roles; the first role present starts at once
  // (its pods still wait for the ConfigMap, as in the reference)
  for (auto& r : api::role_order()) {
    if (!job.spec.role(r)) continue;
    return r != role;
  }
  return false;
}

Value construct_pod(const PaddleJob& job, const std::string& role, int idx, const Options& opt) {
  const api::ResourceSpec* rs = job.spec.role(role);
  const std::string name = res_name(job.name(), role, idx);
  Value pod = Value::object();
  pod["apiVersion"] = "v1";
  pod["kind"] = "Pod";
  Value md = rs ? rs->tmpl.get("metadata") : Value();
  if (!md.is_object()) md = Value::object();
  md.erase("creationTimestamp");
  Value& labels = md["labels"];
  if (!labels.is_object()) labels = Value::object();
  labels[api::kLabelResourceName] = name;
  labels[api::kLabelResourceType] = role;
  Value& ann = md["annotations"];
  if (!ann.is_object()) ann = Value::object();
  ann[api::kAnnotationResource] = role;
  if (start_gated(job, role, opt)) ann[api::kAnnotationStartGate] = api::kGateHold;
  md["name"] = name;
  md["namespace"] = job.ns();
  pod["metadata"] = md;

  Value spec = rs ? rs->tmpl.get("spec") : Value();
  if (!spec.is_object()) spec = Value::object();
  spec["hostname"] = name;
  spec["subdomain"] = name;
  Value& containers = spec["containers"];
  if (!containers.is_array() || containers.size() == 0) {
    pod["spec"] = spec;
    return pod;  // validate() rejects this before a pod is ever created
  }
  Value& c0 = containers[0];
  Value& envs = c0["env"];
  if (!envs.is_array()) envs = Value::array();
  const bool svc = job.spec.intranet == api::intranet::Service;
  {
    Value e = Value::object();
    e["name"] = "POD_IP";
    if (svc) {
      e["value"] = name;
    } else {
      e["valueFrom"]["fieldRef"]["fieldPath"] = "status.podIP";
    }
    envs.push_back(e);
  }
  envs.push_back(env("PADDLE_TRAINER_ID", std::to_string(idx)));
  envs.push_back(env("TRAINING_ROLE", api::training_role(role)));
  envs.push_back(env("PADDLE_TRAINING_ROLE", api::training_role(role)));
  if (job.spec.elastic) {
    envs.push_back(env("PADDLE_ELASTIC_JOB_ID", job.ns() + "-" + job.name()));
    const api::ResourceSpec* w = job.spec.role(api::kRoleWorker);
    envs.push_back(env("PADDLE_ELASTIC_NP", std::to_string(w ? w->replicas : 0)));
    envs.push_back(env("PADDLE_ELASTIC_TIMEOUT", "60"));
  } else {
    Value ef = Value::object();
    ef["configMapRef"]["name"] = job.name();
    Value& efs = c0["envFrom"];
    if (!efs.is_array()) efs = Value::array();
    efs.push_back(ef);
  }
  if (svc) {
    Value p = Value::object();
    p["containerPort"] = api::kPaddlePort;
    Value& ports = c0["ports"];
    if (!ports.is_array()) ports = Value::array();
    ports.push_back(p);
  } else if (job.spec.intranet == api::intranet::Host) {
    spec["hostNetwork"] = true;
  }
  const std::string rp = spec.get("restartPolicy").str();
  if (job.spec.elastic) {
    spec["restartPolicy"] = "OnFailure";
  } else if (rp.empty()) {
    spec["restartPolicy"] = (role == api::kRoleWorker && svc) ? "OnFailure" : "Never";
  }

  // ---- createPod additions (paddlejob_controller.go:234-275)
  if (!opt.init_image.empty()) {
    Value& ic = spec["initContainers"];
    if (!ic.is_array()) ic = Value::array();
    ic.push_back(coord_init_container(opt.init_image));
  }
  if (opt.volcano && !without_volcano(job)) {
    spec["schedulerName"] = kSchedulerVolcano;
    Value& a = md["annotations"];
    a[kPodGroupAnnotation] = job.name();
    a[kVolcanoTaskSpec] = role;
    a[kVolcanoJobName] = job.name();
    a[kVolcanoJobVersion] = std::to_string(job.status.observed_generation);
    a[kVolcanoQueueName] = job.spec.scheduling.present ? job.spec.scheduling.queue : "";
    pod["metadata"] = md;
  }
  if (job.spec.elastic && !opt.etcd_endpoints.empty())
    envs.push_back(env("PADDLE_ELASTIC_SERVER", join(opt.etcd_endpoints, ",")));

  // ---- MI355X additions
  if (opt.launcher_env) {
    const api::ResourceSpec* rr = job.spec.role(role);
    envs.push_back(env("PDO_JOB", job.ns() + "/" + job.name()));
    envs.push_back(env("PDO_ROLE", role));
    envs.push_back(env("PDO_REPLICA_INDEX", std::to_string(idx)));
    envs.push_back(env("PDO_REPLICAS", std::to_string(rr ? rr->replicas : 0)));
  }
  if (opt.gpu_resource_rewrite) {
    for (auto& c : containers.arr()) rewrite_gpu_resources(c);
  }
  pod["spec"] = spec;
  set_controller_reference(pod, job);
  return pod;
}

static bool is_ipv4_like(const std::string& ip) {
  int dots = 0;
  for (char c : ip)
    if (c == '.') ++dots;
  return dots == 3;  // strings.Split(ip, ".") has 4 parts (paddlejob_helper.go:226)
}

Value construct_configmap(const PaddleJob& job, const std::vector<Value>& pods, bool host_port_endpoints) {
  std::map<std::string, std::vector<std::string>> eps;
  for (auto& r : api::role_order()) {
    const api::ResourceSpec* rs = job.spec.role(r);
    if (rs) eps[r] = std::vector<std::string>(rs->replicas > 0 ? rs->replicas : 0);
  }
  const bool svc = job.spec.intranet == api::intranet::Service;
  // D-5: the reference writes :2379 into every endpoint even in Host mode,
  // where the ranks listen on the allocated block (PADDLE_PORT); fast mode
  // advertises the block's base port, compat mode keeps the reference value
  const bool host = job.spec.intranet == api::intranet::Host;
  const std::string hp = host ? job.annotation(api::kAnnotationHostPort) : std::string();
  const int base = host_port_endpoints && !hp.empty() ? std::atoi(hp.c_str()) : api::kPaddlePort;
  const std::string port = std::to_string(base);
  for (auto& pod : pods) {
    const std::string& ip = pod.at_path("status.podIP").as_string();
    if (!is_ipv4_like(ip)) return Value();
    const std::string& pname = pod.at_path("metadata.name").as_string();
    auto ri = extract_name_index(pname);
    auto it = eps.find(ri.first);
    if (it == eps.end() || ri.second < 0 || ri.second >= (int)it->second.size()) continue;  // excess pod
    it->second[ri.second] = (svc ? pname : ip) + ":" + port;
  }
  Value cm = Value::object();
  cm["apiVersion"] = "v1";
  cm["kind"] = "ConfigMap";
  Value& md = cm["metadata"];
  md["name"] = job.name();
  md["namespace"] = job.ns();
  md["labels"][api::kLabelResourceName] = job.name();
  md["annotations"] = Value::object();
  Value& data = cm["data"];
  data["TRAINER_PORTS_NUM"] = std::to_string(api::kPortsPerPod);
  data["PADDLE_PORT"] = host ? hp : port;
  if (job.spec.role(api::kRolePS)) data["PADDLE_PSERVERS_IP_PORT_LIST"] = join(eps[api::kRolePS], ",");
  if (const api::ResourceSpec* w = job.spec.role(api::kRoleWorker)) {
    data["PADDLE_TRAINER_ENDPOINTS"] = join(eps[api::kRoleWorker], ",");
    data["PADDLE_TRAINERS"] = endpoints_to_hosts(eps[api::kRoleWorker]);
    data["PADDLE_TRAINERS_NUM"] = std::to_string(w->replicas);
  }
  if (job.spec.role(api::kRoleHeter)) data["PADDLE_HETER_ENDPOINTS"] = join(eps[api::kRoleHeter], ",");
  auto ps = eps.find(api::kRolePS);
  if (job.spec.with_gloo && *job.spec.with_gloo > 0 && ps != eps.end() && !ps->second.empty()) {
    data["PADDLE_WITH_GLOO"] = std::to_string(*job.spec.with_gloo);
    data["PADDLE_GLOO_RENDEZVOUS"] = "3";
    std::string ep = ps->second[0];
    const std::string from = ":" + port, to = ":" + std::to_string(base + api::kPortsPerPod - 2);
    size_t at = ep.find(from);
    if (at != std::string::npos) ep.replace(at, from.size(), to);
    data["PADDLE_GLOO_HTTP_ENDPOINT"] = ep;
  }
  set_controller_reference(cm, job);
  return cm;
}

Value construct_service_for_pod(const Value& pod) {
  Value svc = Value::object();
  svc["apiVersion"] = "v1";
  svc["kind"] = "Service";
  Value& md = svc["metadata"];
  md["name"] = pod.at_path("metadata.name");
  md["namespace"] = pod.at_path("metadata.namespace");
  md["labels"] = Value::object();
  Value ports = Value::array();
  for (int i = 0; i < api::kPortsPerPod; ++i) {
    Value p = Value::object();
    p["name"] = "p-" + std::to_string(i);
    p["port"] = api::kPaddlePort + i;
    ports.push_back(p);
  }
  svc["spec"]["ports"] = ports;
  svc["spec"]["selector"][api::kLabelResourceName] = pod.at_path("metadata.name");
  svc["spec"]["clusterIP"] = "None";
  return svc;
}

int total_replicas(const PaddleJob& job) {
  int t = 0;
  for (auto& r : api::role_order())
    if (const api::ResourceSpec* rs = job.spec.role(r)) t += rs->replicas;
  return t;
}

Value pg_min_resources(const PaddleJob& job, bool rewrite_gpu) {
  std::vector<std::string> order;
  std::map<std::string, Quantity> tot;
  auto add = [&](const Value& rl) {
    for (auto& m : rl.obj()) {
      Quantity q;
      std::string qs = m.second.is_string() ? m.second.as_string() : m.second.dump();
      if (!Quantity::parse(qs, &q)) continue;
      const std::string key = (rewrite_gpu && m.first == kNVGPU) ? std::string(kAMDGPU) : m.first;
      auto it = tot.find(key);
      if (it == tot.end()) {
        tot[key] = q;
        order.push_back(key);
      } else {
        it->second.add(q);
      }
    }
  };
  for (auto& r : api::role_order()) {
    const api::ResourceSpec* rs = job.spec.role(r);
    if (!rs) continue;
    for (int i = 0; i < rs->replicas; ++i) {
      for (auto& c : rs->tmpl.at_path("spec.containers").arr()) {
        const Value& req = c.at_path("resources.requests");
        if (!req.is_null()) add(req);
        else add(c.at_path("resources.limits"));
      }
    }
  }
  Value out = Value::object();
  for (auto& k : order) out[k] = tot[k].str();
  return out;
}

Value construct_podgroup(const PaddleJob& job, bool rewrite_gpu) {
  Value pg = Value::object();
  pg["apiVersion"] = "scheduling.volcano.sh/v1beta1";
  pg["kind"] = "PodGroup";
  pg["metadata"]["namespace"] = job.ns();
  pg["metadata"]["name"] = job.name();
  Value& spec = pg["spec"];
  spec["minMember"] = total_replicas(job);
  spec["minResources"] = pg_min_resources(job, rewrite_gpu);
  const api::SchedulingPolicy& sp = job.spec.scheduling;
  if (sp.present) {
    if (sp.min_available) spec["minMember"] = *sp.min_available;
    if (!sp.queue.empty()) spec["queue"] = sp.queue;
    if (!sp.priority_class.empty()) spec["priorityClassName"] = sp.priority_class;
    if (sp.min_resources.is_object()) spec["minResources"] = sp.min_resources;
  }
  set_controller_reference(pg, job);
  return pg;
}

}  // namespace build
}  // namespace pdo
