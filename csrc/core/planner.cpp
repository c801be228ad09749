// SPDX-License-Identifier: Apache-2.0
#include "planner.h"

#include <algorithm>
#include <cstdlib>
#include <set>

namespace pdo {
namespace plan {

using api::PaddleJob;

const char* mode_name(Mode m) { return m == Mode::Compat ? "compat" : "fast"; }

const char* op_name(Op op) {
  switch (op) {
    case Op::AddFinalizer: return "AddFinalizer";
    case Op::RemoveFinalizer: return "RemoveFinalizer";
    case Op::SetHostPortAnnotation: return "SetHostPortAnnotation";
    case Op::UpdateStatus: return "UpdateStatus";
    case Op::CreatePodGroup: return "CreatePodGroup";
    case Op::DeletePodGroup: return "DeletePodGroup";
    case Op::CreatePod: return "CreatePod";
    case Op::DeletePod: return "DeletePod";
    case Op::CreateService: return "CreateService";
    case Op::DeleteService: return "DeleteService";
    case Op::CreateConfigMap: return "CreateConfigMap";
    case Op::SyncNP: return "SyncNP";
    case Op::ReleaseRole: return "ReleaseRole";
    case Op::ReleaseGate: return "ReleaseGate";
    case Op::Event: return "Event";
  }
  return "?";
}

Options Options::compat_defaults() {
  Options o;
  o.mode = Mode::Compat;
  o.build.init_image = "docker.io/library/busybox:1";  // main.go:78 default
  o.sync.compat_phase_lag = true;
  o.sync.count_unknown = false;
  o.sync.set_observed_generation = false;
  return o;
}

Options Options::fast_defaults() {
  Options o;
  o.mode = Mode::Fast;
  o.build.init_image = "";
  return o;
}

std::string np_key(const PaddleJob& job) { return "/paddle/" + job.ns() + "-" + job.name() + "/np"; }

static bool has(const std::vector<std::string>& v, const std::string& s) {
  return std::find(v.begin(), v.end(), s) != v.end();
}

static const std::string& obj_name(const Value& o) { return o.at_path("metadata.name").as_string(); }
static bool terminating(const Value& o) { return !o.at_path("metadata.deletionTimestamp").is_null(); }

static Action act(Op op, const std::string& name = "", Value obj = Value()) {
  Action a;
  a.op = op;
  a.name = name;
  a.obj = std::move(obj);
  return a;
}

Plan reconcile(const Observed& obs, const Options& opt, HostPorts* ports, double now) {
  Plan p;
  const bool compat = opt.mode == Mode::Compat;
  PaddleJob job = obs.job;  // mutated as the pass proceeds (status, annotations)

  // ---------------------------------------------------------- 2. finalizer
  {
    auto fins = job.finalizers();
    if (!job.deleting()) {
      if (!has(fins, api::kFinalizer)) p.actions.push_back(act(Op::AddFinalizer, job.name()));
    } else {
      if (has(fins, api::kFinalizer)) {
        if (job.spec.intranet == api::intranet::Host && job.has_annotation(api::kAnnotationHostPort)) {
          int port = atoi(job.annotation(api::kAnnotationHostPort).c_str());
          if (ports && ports->release(port)) {
            p.requeue_after = 1.0;
            p.step = "finalize/release-host-port";
            return p;
          }
        }
        p.actions.push_back(act(Op::RemoveFinalizer, job.name()));
      }
      // the reference continues reconciling a terminating job after removing
      // its finalizer (creating pods the GC then deletes); stop here instead
      p.step = "finalize/deleting";
      return p;
    }
  }

  // ---------------------------------------------------------- 3-4. status
  api::Status ns = fsm::sync_status(job, obs.pods, now, opt.sync);
  p.status = ns;
  if (ns.to_json() != job.status.to_json()) {
    p.status_changed = true;
    p.actions.push_back(act(Op::UpdateStatus, job.name(), ns.to_json()));
  }
  job.status = ns;

  // ---------------------------------------------------------- 5. volcano gate
  if (opt.volcano && !build::without_volcano(job)) {
    const bool terminal = job.status.phase == api::phase::Failed || job.status.phase == api::phase::Completed;
    if (terminal) {
      if (obs.podgroup_exists) {
        p.actions.push_back(act(Op::DeletePodGroup, job.name()));
        p.requeue = true;
        p.step = "volcano/delete-podgroup";
        return p;
      }
    } else if (!obs.podgroup_exists) {
      p.actions.push_back(act(Op::CreatePodGroup, job.name(), build::construct_podgroup(job, opt.build.gpu_resource_rewrite)));
      p.requeue = true;
      p.step = "volcano/create-podgroup";
      return p;
    } else if (obs.podgroup_phase != "Running" && obs.podgroup_phase != "Inqueue") {
      p.requeue = true;
      p.step = "volcano/wait-inqueue";
      return p;
    }
  }

  // ---------------------------------------------------------- 6. scale-in
  {
    bool any = false;
    for (auto& pod : obs.pods) {
      auto ri = build::extract_name_index(obj_name(pod));
      const api::ResourceSpec* rs = job.spec.role(ri.first);
      bool excess = rs && ri.second >= rs->replicas;
      if (!compat && !rs && !ri.first.empty() && build::controller_owner(pod) == job.name()) excess = true;  // D-10
      if (!excess) continue;
      any = true;
      if (!terminating(pod)) p.actions.push_back(act(Op::DeletePod, obj_name(pod)));
      if (compat) break;  // one per pass; a terminating pod still ends the pass (D-4)
    }
    if (any) {
      p.requeue = true;
      p.step = "scale-in";
      return p;
    }
  }

  // ---------------------------------------------------------- 7. services
  if (job.spec.intranet == api::intranet::Service) {
    std::set<std::string> have;
    for (auto& s : obs.services) have.insert(obj_name(s));
    for (auto& pod : obs.pods) {
      if (have.count(obj_name(pod))) continue;
      Value svc = build::construct_service_for_pod(pod);
      build::set_controller_reference(svc, job);
      p.actions.push_back(act(Op::CreateService, obj_name(pod), svc));
      if (compat) {
        p.step = "service/create";
        return p;
      }
    }
    // fast mode: the reference leaves the Service of a scaled-in pod behind
    // until the job is cleaned up (paddlejob_controller.go:161-191); drop it
    if (!compat) {
      for (auto& s : obs.services) {
        auto ri = build::extract_name_index(obj_name(s));
        const api::ResourceSpec* rs = job.spec.role(ri.first);
        if (rs && ri.second >= rs->replicas && !terminating(s))
          p.actions.push_back(act(Op::DeleteService, obj_name(s)));
      }
    }
  }

  // ---------------------------------------------------------- 8. host ports
  if (job.spec.intranet == api::intranet::Host && ports) {
    if (job.has_annotation(api::kAnnotationHostPort)) {
      int port = atoi(job.annotation(api::kAnnotationHostPort).c_str());
      if (!ports->registered(port) && !job.deleting()) {
        ports->register_port(port);  // controller restarted: re-learn the allocation
        if (compat) {
          p.requeue_after = 1.0;
          p.step = "hostport/register";
          return p;
        }
      }
    } else {
      const int port = ports->allocate();
      Action a = act(Op::SetHostPortAnnotation, job.name());
      a.detail = std::to_string(port);
      p.actions.push_back(a);
      job.metadata["annotations"][api::kAnnotationHostPort] = a.detail;
      if (compat) {
        p.requeue_after = 1.0;
        p.step = "hostport/allocate";
        return p;
      }
    }
  }

  // ---------------------------------------------------------- 9. elastic np
  if (job.spec.elastic && opt.kv) {
    if (!obs.kv_ok) {
      p.requeue = true;
      p.step = "elastic/kv-error";
      return p;
    }
    const api::ResourceSpec* w = job.spec.role(api::kRoleWorker);
    if (job.status.mode == api::mode::Collective && w) {
      const std::string np = std::to_string(w->replicas);
      if (obs.kv_count == 1 && obs.kv_np != np) {
        Action a = act(Op::SyncNP, np_key(job));
        a.detail = np;
        p.actions.push_back(a);
        Action ev = act(Op::Event, job.name());
        ev.role = "Normal";
        ev.detail = "Scaled";
        ev.obj = Value("scaled replicas to " + np);
        p.actions.push_back(ev);
        p.requeue = true;
        p.step = "elastic/scaled";
        return p;
      }
    }
  }

  // ---------------------------------------------------------- 10-11. cleanup
  {
    const std::string& ph = job.status.phase;
    const std::string& pol = job.spec.clean_pod_policy;
    bool clean = false;
    if (ph == api::phase::Failed && (pol == api::clean::Always || pol == api::clean::OnFailure)) clean = true;
    if (ph == api::phase::Completed &&
        (pol.empty() || pol == api::clean::Always || pol == api::clean::OnCompletion))
      clean = true;
    if (clean) {
      if (compat) {
        // cleanOne: first pod (skipped if terminating), else first service
        if (!obs.pods.empty()) {
          if (!terminating(obs.pods[0])) p.actions.push_back(act(Op::DeletePod, obj_name(obs.pods[0])));
        } else if (!obs.services.empty()) {
          if (!terminating(obs.services[0])) p.actions.push_back(act(Op::DeleteService, obj_name(obs.services[0])));
        }
      } else {
        for (auto& pod : obs.pods)
          if (!terminating(pod)) p.actions.push_back(act(Op::DeletePod, obj_name(pod)));
        for (auto& s : obs.services)
          if (!terminating(s)) p.actions.push_back(act(Op::DeleteService, obj_name(s)));
      }
      p.step = "cleanup";
      return p;
    }
  }

  // ---------------------------------------------------------- 12. create pods
  {
    std::set<std::string> existing;
    for (auto& pod : obs.pods) existing.insert(obj_name(pod));
    bool created = false;
    build::Options bopt = opt.build;
    bopt.volcano = opt.volcano;  // --scheduling=volcano also stamps schedulerName + group annotations
    for (auto& role : api::role_order()) {
      const api::ResourceSpec* rs = job.spec.role(role);
      const api::ResourceStatus* st = job.status.role(role);
      const bool done = !rs || (st && (int)st->refs.size() == rs->replicas);
      if (done) continue;
      for (int i = 0; i < rs->replicas; ++i) {
        const std::string name = build::res_name(job.name(), role, i);
        if (existing.count(name)) continue;
        Action a = act(Op::CreatePod, name, build::construct_pod(job, role, i, bopt));
        a.role = role;
        p.actions.push_back(a);
        created = true;
        if (compat) {
          p.step = "pods/create";
          return p;
        }
      }
    }
    if (created) {
      // fast: the ConfigMap needs pod IPs, which only arrive with later events
      p.step = "pods/create";
      return p;
    }
  }

  // ---------------------------------------------------------- 13. configmap
  if (!job.spec.elastic && fsm::all_pods_ready(job, obs.pods) && !obs.configmap_exists) {
    Value cm = build::construct_configmap(job, obs.pods, /*host_port_endpoints=*/!compat);
    if (cm.is_null()) {
      p.requeue = true;
      p.step = "configmap/wait-ipv4";
      return p;
    }
    p.actions.push_back(act(Op::CreateConfigMap, job.name(), cm));
    p.step = "configmap/create";
    return p;
  }

  // ---------------------------------------------- 14a. native start gate (fast)
  // Same order as the coordinator below (ps → worker → heter, a role released
  // once every earlier role is fully Running), but event-driven: a pod status
  // change re-runs the pass, no 1 s requeue, no exec.
  if (!compat && opt.build.start_gate && opt.build.init_image.empty()) {
    bool earlier_running = true;
    for (auto& role : api::role_order()) {
      const api::ResourceSpec* rs = job.spec.role(role);
      if (!rs) continue;
      Action a = act(Op::ReleaseGate, role);
      a.role = role;
      for (auto& pod : obs.pods) {
        if (pod.at_path("metadata.annotations").get(api::kAnnotationResource).as_string() == role &&
            pod.at_path("metadata.annotations").get(api::kAnnotationStartGate).as_string() == api::kGateHold &&
            pod.at_path("metadata.deletionTimestamp").is_null())
          a.targets.push_back(obj_name(pod));
      }
      if (!a.targets.empty()) {
        if (!earlier_running) {
          p.step = "gate/wait-" + role;
          return p;
        }
        p.actions.push_back(a);
        p.step = "gate/release-" + role;
        return p;
      }
      const api::ResourceStatus* st = job.status.role(role);
      if (!st || st->running < rs->replicas) earlier_running = false;
    }
  }

  // ---------------------------------------------------------- 14. coordinator
  if (job.status.phase == api::phase::Starting && !opt.build.init_image.empty()) {
    const auto& order = api::role_order();
    for (size_t i = 0; i < order.size(); ++i) {
      const api::ResourceStatus* st = job.status.role(order[i]);
      const api::ResourceSpec* rs = job.spec.role(order[i]);
      if (!st || !rs || st->running >= rs->replicas) continue;
      if (i == 0 && st->running == 0 && !fsm::all_coord_running(obs.pods)) {
        p.requeue_after = compat ? 1.0 : 0.1;
        p.step = "coordinator/wait-all-init";
        return p;
      }
      Action a = act(Op::ReleaseRole, order[i]);
      a.role = order[i];
      for (auto& pod : obs.pods) {
        if (pod.at_path("metadata.annotations").get(api::kAnnotationResource).as_string() == order[i] &&
            fsm::coord_running(pod))
          a.targets.push_back(obj_name(pod));
      }
      p.actions.push_back(a);
      p.requeue_after = compat ? 1.0 : 0.1;
      p.step = "coordinator/release-" + order[i];
      return p;
    }
  }
  p.step = "done";
  return p;
}

}  // namespace plan
}  // namespace pdo
