// SPDX-License-Identifier: Apache-2.0
#include "status.h"

#include "builders.h"

namespace pdo {
namespace fsm {

using api::PaddleJob;
using api::ResourceSpec;
using api::ResourceStatus;

bool pod_really_running(const Value& pod) {
  if (pod.at_path("status.phase").as_string() != "Running") return false;
  for (auto& c : pod.at_path("status.initContainerStatuses").arr())
    if (!c.get("ready").as_bool()) return false;
  for (auto& c : pod.at_path("status.containerStatuses").arr()) {
    if (!c.get("ready").as_bool()) return false;
    if (c.at_path("state.running").is_null()) return false;
  }
  return true;
}

bool coord_running(const Value& pod) {
  if (pod.at_path("status.phase").as_string() != "Pending") return false;
  for (auto& c : pod.at_path("status.initContainerStatuses").arr())
    if (c.get("name").as_string() == build::kCoordContainer && !c.at_path("state.running").is_null()) return true;
  return false;
}

bool all_coord_running(const std::vector<Value>& pods) {
  for (auto& p : pods)
    if (!coord_running(p)) return false;
  return true;
}

static bool pod_created(const ResourceSpec* spec, const ResourceStatus* st) {
  if (!spec) return true;
  return st && (int)st->refs.size() == spec->replicas;
}

bool all_pods_created(const PaddleJob& job) {
  for (auto& r : api::role_order())
    if (!pod_created(job.spec.role(r), job.status.role(r))) return false;
  return true;
}

bool all_pods_ready(const PaddleJob& job, const std::vector<Value>& pods) {
  if (!all_pods_created(job)) return false;
  for (auto& p : pods)
    if (p.at_path("status.podIP").as_string().empty()) return false;
  return true;
}

std::string derive_phase(const PaddleJob& job) {
  const std::string& cur = job.status.phase;
  if (cur == api::phase::Completed) return api::phase::Completed;
  if (cur == api::phase::Failed) return api::phase::Failed;
  const auto& order = api::role_order();
  auto any = [&](auto pred) {
    for (auto& r : order) {
      const ResourceStatus* st = job.status.role(r);
      if (st && pred(*st)) return true;
    }
    return false;
  };
  if (any([](const ResourceStatus& s) { return s.failed > 0; })) return api::phase::Failed;
  if (any([](const ResourceStatus& s) { return s.starting > 0; })) return api::phase::Starting;
  if (any([](const ResourceStatus& s) { return s.pending > 0; })) return api::phase::Pending;
  // checkAll iterates the *status* map, whose keys are always ps/worker/heter
  auto all = [&](auto pred) {
    for (auto& r : order) {
      const ResourceSpec* sp = job.spec.role(r);
      const ResourceStatus* st = job.status.role(r);
      if (!(sp == nullptr || (st && pred(*sp, *st)))) return false;
    }
    return true;
  };
  if (all([](const ResourceSpec& sp, const ResourceStatus& st) { return sp.replicas == st.running; }))
    return api::phase::Running;
  if (all([](const ResourceSpec& sp, const ResourceStatus& st) { return sp.replicas == st.succeeded; }))
    return api::phase::Completed;
  if (cur.empty()) return api::phase::Pending;
  return cur;
}

std::string derive_mode(const api::Spec& spec) {
  if (spec.role(api::kRolePS)) return api::mode::PS;
  const ResourceSpec* w = spec.role(api::kRoleWorker);
  if (w && w->replicas > 1) return api::mode::Collective;
  return api::mode::Single;
}

static std::string start_time(const api::Status& st, double now) {
  if (st.start_time.empty() && st.phase == api::phase::Running) return api::rfc3339(now);
  return st.start_time;
}

static std::string completion_time(const api::Status& st, double now) {
  if (st.completion_time.empty() && (st.phase == api::phase::Completed || st.phase == api::phase::Failed))
    return api::rfc3339(now);
  return st.completion_time;
}

static void count_pods(api::Status& st, const std::vector<Value>& pods, bool count_unknown) {
  for (auto& pod : pods) {
    const std::string role = pod.at_path("metadata.annotations").get(api::kAnnotationResource).str();
    ResourceStatus* rs = st.role(role);
    if (!rs) continue;
    rs->present = true;
    const std::string& ph = pod.at_path("status.phase").as_string();
    if (ph == "Pending") {
      // held at the start barrier (coordinator init container, or the native gate
      // once the pod has its IP) counts as starting, as paddlejob_controller.go:344-346
      if (coord_running(pod) || (!pod.at_path("status.podIP").as_string().empty() &&
                                 pod.at_path("metadata.annotations").get(api::kAnnotationStartGate).as_string() ==
                                     api::kGateHold))
        rs->starting++;
      else rs->pending++;
    } else if (ph == "Running") {
      if (pod_really_running(pod)) rs->running++;
      else rs->starting++;
    } else if (ph == "Failed") {
      rs->failed++;
    } else if (ph == "Succeeded") {
      rs->succeeded++;
    } else if (count_unknown && ph == "Unknown") {
      rs->unknown++;
    }
    rs->refs.push_back(build::object_reference(pod, "v1", "Pod"));
  }
}

api::Status sync_status(const PaddleJob& job, const std::vector<Value>& pods, double now, const SyncOptions& opt) {
  api::Status st;
  if (opt.compat_phase_lag) {
    // reference order: phase/mode/times from the OLD status, then new counts
    st.phase = derive_phase(job);
    st.mode = derive_mode(job.spec);
    st.start_time = start_time(job.status, now);
    st.completion_time = completion_time(job.status, now);
    count_pods(st, pods, opt.count_unknown);
  } else {
    count_pods(st, pods, opt.count_unknown);
    PaddleJob tmp;
    tmp.spec = job.spec;
    tmp.status = st;
    tmp.status.phase = job.status.phase;  // terminal phases stay terminal
    st.phase = derive_phase(tmp);
    st.mode = derive_mode(job.spec);
    api::Status with_new_phase = job.status;
    with_new_phase.phase = st.phase;
    st.start_time = start_time(with_new_phase, now);
    st.completion_time = completion_time(with_new_phase, now);
  }
  st.elastic = job.status.elastic;
  if (opt.set_observed_generation) st.observed_generation = job.generation();
  return st;
}

}  // namespace fsm
}  // namespace pdo
