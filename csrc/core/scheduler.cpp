// SPDX-License-Identifier: Apache-2.0
#include "scheduler.h"

#include <algorithm>
#include <cstdlib>

#include "builders.h"
#include "log.h"
#include "quantity.h"

namespace pdo {

using json::Value;

int pod_gpu_request(const Value& pod) {
  int total = 0;
  for (auto& c : pod.at_path("spec.containers").arr()) {
    const Value& lim = c.at_path("resources.limits").get(build::kAMDGPU);
    const Value& req = c.at_path("resources.requests").get(build::kAMDGPU);
    const Value& q = lim.is_null() ? req : lim;
    if (q.is_null()) continue;
    Quantity qq;
    if (Quantity::parse(q.is_string() ? q.as_string() : q.dump(), &qq)) total += (int)(qq.milli() / 1000);
  }
  return total;
}

static bool active(const Value& pod) {
  const std::string& ph = pod.at_path("status.phase").as_string();
  return ph != "Succeeded" && ph != "Failed";
}

std::map<std::string, int> Scheduler::free_gpus() const {
  std::map<std::string, int> fr;
  std::map<std::string, int> pods;
  for (auto& n : nodes_) fr[n.name] = n.gpus;
  for (auto& p : s_->list("Pod")) {
    const std::string& nn = p.at_path("spec.nodeName").as_string();
    if (nn.empty() || !fr.count(nn) || !active(p)) continue;
    fr[nn] -= pod_gpu_request(p);
  }
  return fr;
}

bool Scheduler::bind(Value pod, const std::string& node) {
  pod["spec"]["nodeName"] = node;
  try {
    Value cur = s_->update("Pod", pod);
    Value st = cur;
    Value cond = Value::object();
    cond["type"] = "PodScheduled";
    cond["status"] = "True";
    Value& conds = st["status"]["conditions"];
    if (!conds.is_array()) conds = Value::array();
    conds.push_back(cond);
    if (st.at_path("status.phase").is_null()) st["status"]["phase"] = "Pending";
    s_->update_status("Pod", st);
    return true;
  } catch (const store::ApiError&) {
    return false;  // raced with a delete/update: retried next pass
  }
}

int Scheduler::sync() {
  int bound = 0;
  auto fr = free_gpus();
  auto fits = [&](int need) -> std::string {
    for (auto& n : nodes_)
      if (fr[n.name] >= need) return n.name;
    return "";
  };
  int cluster_free = 0;
  for (auto& kv : fr) cluster_free += kv.second;

  // --- gang admission of PodGroups
  std::map<std::string, Value> groups;  // ns/name → pg
  for (auto& pg : s_->list("PodGroup")) {
    const std::string key = pg.at_path("metadata.namespace").str() + "/" + pg.at_path("metadata.name").str();
    std::string phase = pg.at_path("status.phase").str();
    if (phase.empty() || phase == "Pending") {
      Quantity need;
      const Value& mr = pg.at_path("spec.minResources").get(build::kAMDGPU);
      int gpus = 0;
      if (!mr.is_null() && Quantity::parse(mr.is_string() ? mr.as_string() : mr.dump(), &need))
        gpus = (int)(need.milli() / 1000);
      if (gpus <= cluster_free) {
        Value st = pg;
        st["status"]["phase"] = "Inqueue";
        try {
          pg = s_->update_status("PodGroup", st);
        } catch (const store::ApiError&) {
        }
      } else if (phase.empty()) {
        Value st = pg;
        st["status"]["phase"] = "Pending";
        try {
          pg = s_->update_status("PodGroup", st);
        } catch (const store::ApiError&) {
        }
      }
    }
    groups[key] = pg;
  }

  // --- pending pods, creation order
  std::vector<Value> pending;
  for (auto& p : s_->list("Pod")) {
    if (!p.at_path("spec.nodeName").as_string().empty()) continue;
    if (!p.at_path("metadata.deletionTimestamp").is_null()) continue;
    pending.push_back(p);
  }
  std::stable_sort(pending.begin(), pending.end(), [](const Value& a, const Value& b) {
    return atoll(a.at_path("metadata.resourceVersion").as_string().c_str()) <
           atoll(b.at_path("metadata.resourceVersion").as_string().c_str());
  });

  std::map<std::string, std::vector<Value>> gang;  // group key → its pending pods
  for (auto& p : pending) {
    const bool volcano = p.at_path("spec.schedulerName").as_string() == build::kSchedulerVolcano;
    const std::string grp = p.at_path("metadata.annotations").get(build::kPodGroupAnnotation).str();
    if (volcano && !grp.empty()) {
      gang[p.at_path("metadata.namespace").str() + "/" + grp].push_back(p);
      continue;
    }
    const int need = pod_gpu_request(p);
    std::string node = fits(need);
    if (node.empty()) continue;
    if (bind(p, node)) {
      fr[node] -= need;
      ++bound;
    }
  }

  for (auto& g : gang) {
    auto it = groups.find(g.first);
    if (it == groups.end()) continue;  // PodGroup not created yet
    const std::string phase = it->second.at_path("status.phase").str();
    if (phase != "Inqueue" && phase != "Running") continue;
    // all-or-nothing placement of the whole pending set (≥ minMember)
    auto trial = fr;
    std::vector<std::pair<Value, std::string>> plan;
    bool ok = true;
    for (auto& p : g.second) {
      const int need = pod_gpu_request(p);
      std::string node;
      for (auto& n : nodes_)
        if (trial[n.name] >= need) {
          node = n.name;
          break;
        }
      if (node.empty()) {
        ok = false;
        break;
      }
      trial[node] -= need;
      plan.emplace_back(p, node);
    }
    if (!ok) continue;
    for (auto& pn : plan)
      if (bind(pn.first, pn.second)) ++bound;
    fr = trial;
  }

  // --- PodGroup Running / status counts
  for (auto& g : groups) {
    Value pg = g.second;
    const std::string ns = pg.at_path("metadata.namespace").str();
    const std::string name = pg.at_path("metadata.name").str();
    int running = 0, succeeded = 0, failed = 0;
    for (auto& p : s_->list("Pod", ns)) {
      if (p.at_path("metadata.annotations").get(build::kPodGroupAnnotation).as_string() != name) continue;
      const std::string& ph = p.at_path("status.phase").as_string();
      if (ph == "Running") ++running;
      else if (ph == "Succeeded") ++succeeded;
      else if (ph == "Failed") ++failed;
    }
    Value st = pg;
    const int min_member = (int)pg.at_path("spec.minMember").as_int(1);
    std::string phase = pg.at_path("status.phase").str();
    if ((phase == "Inqueue" || phase == "Running") && running + succeeded >= min_member) phase = "Running";
    st["status"]["phase"] = phase;
    if (running) st["status"]["running"] = running;
    else st["status"].erase("running");
    if (succeeded) st["status"]["succeeded"] = succeeded;
    else st["status"].erase("succeeded");
    if (failed) st["status"]["failed"] = failed;
    else st["status"].erase("failed");
    if (!(st.get("status") == pg.get("status"))) {
      try {
        s_->update_status("PodGroup", st);
      } catch (const store::ApiError&) {
      }
    }
  }
  return bound;
}

}  // namespace pdo
