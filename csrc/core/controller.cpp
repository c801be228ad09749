// SPDX-License-Identifier: Apache-2.0
#include "controller.h"

#include <chrono>
#include <cstdio>
#include <random>

#include "builders.h"
#include "log.h"
#include "metrics.h"

namespace pdo {

using json::Value;

static const char* kLogger = "controllers.PaddleJob";

Controller::Controller(store::Store* cache, ObjectApi* api, kv::Client* kv, HostPorts* ports, ExecFn exec,
                       ControllerOptions opt, api::Clock clock)
    : cache_(cache), api_(api), kv_(kv), ports_(ports), exec_(std::move(exec)), opt_(std::move(opt)),
      clock_(clock), q_(clock) {
  auto& m = Metrics::global();
  m.help("controller_runtime_reconcile_total", "counter", "Total number of reconciliations per controller");
  m.help("controller_runtime_reconcile_errors_total", "counter", "Total number of reconciliation errors");
  m.help("controller_runtime_reconcile_time_seconds", "histogram", "Length of time per reconciliation");
  m.help("workqueue_depth", "gauge", "Current depth of workqueue");
  m.help("workqueue_adds_total", "counter", "Total number of adds handled by workqueue");
  m.help("pdo_reconcile_actions_total", "counter", "Mutations applied by the PaddleJob reconciler, by kind");
  m.help("pdo_job_phase_transition_seconds", "histogram",
         "Seconds from PaddleJob creation to each observed phase transition");
  m.help("pdo_job_ready_seconds", "histogram", "Seconds from PaddleJob creation to phase Running");
}

Controller::~Controller() { stop(); }

void Controller::on_event(const store::WatchEvent& ev) {
  const Value& md = ev.object.get("metadata");
  const std::string ns = md.get("namespace").str();
  if (!opt_.watch_namespace.empty() && ns != opt_.watch_namespace) return;
  std::string name;
  if (ev.kind == api::kKind) {
    name = md.get("name").str();
  } else if (ev.kind == "Pod" || ev.kind == "Service" || ev.kind == "ConfigMap" ||
             (ev.kind == "PodGroup" && opt_.plan.volcano)) {
    name = build::controller_owner(ev.object);
  }
  if (name.empty()) return;
  q_.add(ns + "/" + name);
  Metrics::global().inc("workqueue_adds_total", {{"name", "paddlejob"}});
}

bool Controller::process_one(double timeout_s) {
  std::string key;
  if (!q_.get(&key, timeout_s)) return false;
  const size_t slash = key.find('/');
  const std::string ns = key.substr(0, slash), name = key.substr(slash + 1);
  const auto t0 = std::chrono::steady_clock::now();
  ReconcileResult r;
  try {
    r = reconcile(ns, name);
  } catch (const std::exception& e) {
    r.error = true;
    r.message = e.what();
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  auto& m = Metrics::global();
  m.observe("controller_runtime_reconcile_time_seconds", {{"controller", "paddlejob"}}, dt);
  std::string result;
  if (r.error) {
    q_.add_rate_limited(key);
    result = "error";
    m.inc("controller_runtime_reconcile_errors_total", {{"controller", "paddlejob"}});
    log::error(kLogger, "Reconciler error", {{"paddlejob", key}, {"error", r.message}});
  } else if (r.requeue_after > 0) {
    q_.forget(key);
    q_.add_after(key, r.requeue_after);
    result = "requeue_after";
  } else if (r.requeue) {
    q_.add_rate_limited(key);
    result = "requeue";
  } else {
    q_.forget(key);
    result = "success";
  }
  m.inc("controller_runtime_reconcile_total", {{"controller", "paddlejob"}, {"result", result}});
  m.set("workqueue_depth", {{"name", "paddlejob"}}, (double)q_.len());
  q_.done(key);
  return true;
}

void Controller::record_event(const Value& obj, const std::string& kind, const std::string& type,
                              const std::string& reason, const std::string& msg) {
  if (!opt_.record_events) return;
  thread_local std::mt19937_64 rng(std::random_device{}());  // one per worker thread (TSan-clean)
  const Value& md = obj.get("metadata");
  Value ev = Value::object();
  ev["apiVersion"] = "v1";
  ev["kind"] = "Event";
  char suffix[24];
  snprintf(suffix, sizeof suffix, "%016llx", (unsigned long long)rng());
  ev["metadata"]["name"] = md.get("name").str() + "." + suffix;
  ev["metadata"]["namespace"] = md.get("namespace");
  Value io = Value::object();
  io["kind"] = kind;
  io["namespace"] = md.get("namespace");
  io["name"] = md.get("name");
  io["uid"] = md.get("uid");
  io["apiVersion"] = kind == api::kKind ? api::kAPIVersion : "v1";
  io["resourceVersion"] = md.get("resourceVersion");
  ev["involvedObject"] = io;
  ev["reason"] = reason;
  ev["message"] = msg;
  ev["type"] = type;
  ev["source"]["component"] = "paddlejob-controller";
  const std::string ts = api::rfc3339(clock_());
  ev["firstTimestamp"] = ts;
  ev["lastTimestamp"] = ts;
  ev["count"] = 1;
  ev["reportingComponent"] = "paddlejob-controller";
  try {
    api_->create("Event", ev);
  } catch (const std::exception&) {
    // events are best effort (EventRecorder semantics)
  }
}

static bool is_conflict(const store::ApiError& e) { return e.code == store::ApiError::Conflict; }

void Controller::apply(const api::PaddleJob& job, Value raw, const plan::Plan& p, ReconcileResult* r) {
  using plan::Op;
  const std::string ns = job.ns();
  auto& m = Metrics::global();
  for (const plan::Action& a : p.actions) {
    m.inc("pdo_reconcile_actions_total", {{"kind", plan::op_name(a.op)}});
    r->actions++;
    try {
      switch (a.op) {
        case Op::AddFinalizer:
        case Op::RemoveFinalizer: {
          Value& fins = raw["metadata"]["finalizers"];
          if (a.op == Op::AddFinalizer) {
            if (!fins.is_array()) fins = Value::array();
            fins.push_back(api::kFinalizer);
          } else {
            Value keep = Value::array();
            for (auto& f : fins.arr())
              if (f.as_string() != api::kFinalizer) keep.push_back(f);
            if (keep.size()) fins = keep;
            else raw["metadata"].erase("finalizers");
          }
          raw = api_->update(api::kKind, raw);
          break;
        }
        case Op::SetHostPortAnnotation: {
          raw["metadata"]["annotations"][api::kAnnotationHostPort] = a.detail;
          raw = api_->update(api::kKind, raw);
          break;
        }
        case Op::UpdateStatus: {
          Value st = raw;
          st["status"] = a.obj;
          raw = api_->update_status(api::kKind, st);
          break;
        }
        case Op::CreatePod:
        case Op::CreateService:
        case Op::CreateConfigMap:
        case Op::CreatePodGroup: {
          const std::string kind = a.op == Op::CreatePod ? "Pod" : a.op == Op::CreateService ? "Service"
                                   : a.op == Op::CreateConfigMap ? "ConfigMap" : "PodGroup";
          try {
            api_->create(kind, a.obj);
            record_event(raw, api::kKind, "Normal", "Created", "created " + kind + " " + a.name);
          } catch (const store::ApiError& e) {
            if (e.code == store::ApiError::AlreadyExists) break;  // cache lag: already there
            record_event(raw, api::kKind, "Warning", "Create", "create failed " + kind + " " + a.name);
            throw;
          }
          break;
        }
        case Op::DeletePod:
        case Op::DeleteService:
        case Op::DeletePodGroup: {
          const std::string kind = a.op == Op::DeletePod ? "Pod" : a.op == Op::DeleteService ? "Service" : "PodGroup";
          try {
            api_->remove(kind, ns, a.name, kind == "Pod" && opt_.graceful_pod_delete);
            record_event(raw, api::kKind, "Normal", "Deleted", "deleted " + kind + " " + a.name);
          } catch (const store::ApiError& e) {
            if (e.code == store::ApiError::NotFound) break;
            record_event(raw, api::kKind, "Warning", "Delete", "delete failed " + kind + " " + a.name);
            throw;
          }
          break;
        }
        case Op::SyncNP: {
          if (!kv_ || !kv_->put(a.name, a.detail)) {
            r->error = true;
            r->message = "sync np failed";
            return;
          }
          log::info(kLogger, "Scaled", {{"new replicas", a.detail}});
          break;
        }
        case Op::ReleaseRole: {
          for (auto& pod : a.targets)
            if (exec_) exec_(ns, pod, build::kCoordContainer, {"touch", "goon"});
          break;
        }
        case Op::ReleaseGate: {
          for (auto& pod : a.targets) {
            Value obj;
            if (!cache_->try_get("Pod", ns, pod, &obj)) continue;
            obj["metadata"]["annotations"][api::kAnnotationStartGate] = api::kGateReleased;
            try {
              api_->update("Pod", obj);
            } catch (const store::ApiError& e) {
              if (e.code == store::ApiError::NotFound) continue;
              throw;  // conflict: requeue, the next pass re-lists the held pods
            }
          }
          break;
        }
        case Op::Event: {
          record_event(raw, api::kKind, a.role.empty() ? "Normal" : a.role, a.detail, a.obj.str());
          break;
        }
      }
    } catch (const store::ApiError& e) {
      if (is_conflict(e)) {
        r->requeue_after = 1.0;  // paddlejob_controller.go:113,127
        r->requeue = false;
        r->message = e.what();
        return;
      }
      r->error = true;
      r->message = e.what();
      return;
    }
  }
}

ReconcileResult Controller::reconcile(const std::string& ns, const std::string& name) {
  ReconcileResult r;
  Value raw;
  if (!cache_->try_get(api::kKind, ns, name, &raw)) {
    std::lock_guard<std::mutex> g(meta_mu_);
    last_phase_.erase(ns + "/" + name);
    first_seen_.erase(ns + "/" + name);
    return r;  // IgnoreNotFound
  }
  api::PaddleJob job = api::PaddleJob::from_json(raw);
  log::debug(kLogger, "Reconcile", {{"version", raw.at_path("metadata.resourceVersion").str()},
                                    {"phase", job.status.phase},
                                    {"delete", raw.at_path("metadata.deletionTimestamp").str()}});
  auto errs = api::validate(job);
  if (!errs.empty() && !job.deleting()) {
    std::string msg;
    for (auto& e : errs) msg += e + "; ";
    record_event(raw, api::kKind, "Warning", "Invalid", msg);
    r.message = msg;
    return r;  // do not requeue an invalid spec until it changes
  }

  plan::Observed obs;
  obs.job = job;
  obs.pods = cache_->list("Pod", ns, {}, name);
  if (job.spec.intranet == api::intranet::Service) obs.services = cache_->list("Service", ns, {}, name);
  obs.configmap_exists = cache_->try_get("ConfigMap", ns, name, nullptr);
  if (opt_.plan.volcano) {
    Value pg;
    obs.podgroup_exists = cache_->try_get("PodGroup", ns, name, &pg);
    if (obs.podgroup_exists) obs.podgroup_phase = pg.at_path("status.phase").str();
  }
  if (job.spec.elastic && kv_ && opt_.plan.kv) {
    std::vector<kv::KeyValue> kvs;
    obs.kv_ok = kv_->get(plan::np_key(job), &kvs);
    obs.kv_count = (int)kvs.size();
    if (!kvs.empty()) obs.kv_np = kvs[0].value;
  }
  const double now = clock_();
  plan::Plan p = plan::reconcile(obs, opt_.plan, ports_, now);
  r.step = p.step;
  r.requeue = p.requeue;
  r.requeue_after = p.requeue_after;
  apply(job, raw, p, &r);

  // phase-transition metrics
  const std::string key = ns + "/" + name;
  const std::string newp = p.status.phase;
  std::lock_guard<std::mutex> g(meta_mu_);
  const std::string oldp = last_phase_[key];
  if (!newp.empty() && newp != oldp && !job.deleting()) {
    const double created = api::parse_rfc3339(raw.at_path("metadata.creationTimestamp").str());
    const double age = created > 0 ? now - created : 0;
    Metrics::global().observe("pdo_job_phase_transition_seconds", {{"from", oldp}, {"to", newp}}, age);
    if (newp == api::phase::Running) Metrics::global().observe("pdo_job_ready_seconds", {}, age);
    last_phase_[key] = newp;
  }
  return r;
}

void Controller::start() {
  if (running_.exchange(true)) return;
  for (int i = 0; i < std::max(1, opt_.workers); ++i)
    workers_.emplace_back([this] {
      while (running_) process_one(0.05);
    });
}

void Controller::stop() {
  if (!running_.exchange(false)) return;
  q_.shutdown();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
}

}  // namespace pdo
