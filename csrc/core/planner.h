// SPDX-License-Identifier: Apache-2.0
// Reconcile planner: observed state → ordered action list (+ requeue hint).
//
// The reference Reconcile (controllers/paddlejob_controller.go:101-333)
// interleaves decisions with API calls and returns after (at most) one
// mutation.  Here the decision logic is a deterministic function so it can be
// unit-tested without any cluster, and one planner serves two execution modes:
//
//  * Mode::Compat reproduces the reference sequencing step by step (SURVEY
//    §3.2 table): one object mutation per pass, the same early returns and
//    1 s requeues, ConfigMap barrier, ps→worker→heter coordinator release,
//    one-pass phase lag (D-2).  Used as the on-hardware baseline.
//  * Mode::Fast keeps every observable outcome (objects, env contract,
//    status schema) but batches creates/deletes in one pass, derives the
//    phase from the current counts, cleans pods of removed roles (D-10),
//    refreshes nothing it does not need to, and never polls on a timer where
//    an event will arrive.
//
// The executor (controller.cpp) applies actions in order and stops at the
// first failure (an API error requeues with backoff, as controller-runtime).
#pragma once

#include <string>
#include <vector>

#include "api.h"
#include "builders.h"
#include "hostport.h"
#include "status.h"

namespace pdo {
namespace plan {

using json::Value;

enum class Mode { Compat, Fast };
const char* mode_name(Mode m);

enum class Op {
  AddFinalizer,
  RemoveFinalizer,
  SetHostPortAnnotation,
  UpdateStatus,
  CreatePodGroup,
  DeletePodGroup,
  CreatePod,
  DeletePod,
  CreateService,
  DeleteService,
  CreateConfigMap,
  SyncNP,       // elastic: put /paddle/<ns>-<name>/np
  ReleaseRole,  // coordinator: `touch goon` in the coord container of these pods
  ReleaseGate,  // native barrier: set the start-gate annotation of these pods to "released"
  Event,
};
const char* op_name(Op op);

struct Action {
  Op op;
  std::string name;    // object name (pod/service/...) or KV key
  std::string role;    // for ReleaseRole / CreatePod
  std::string detail;  // event reason / kv value / annotation value
  Value obj;           // object to create / status to write
  std::vector<std::string> targets;  // ReleaseRole: pod names
};

struct Observed {
  api::PaddleJob job;
  std::vector<Value> pods;      // children (owner index)
  std::vector<Value> services;  // children (only listed in Service mode)
  bool configmap_exists = false;
  bool podgroup_exists = false;
  std::string podgroup_phase;   // Pending / Inqueue / Running / Unknown
  // elastic KV (`np` key); kv_ok=false → the KV read failed
  bool kv_ok = true;
  int kv_count = 0;             // number of kvs under the key (reference requires exactly 1)
  std::string kv_np;
};

struct Options {
  Mode mode = Mode::Fast;
  build::Options build;
  bool volcano = false;  // --scheduling=volcano
  bool kv = false;       // --etcd-server configured
  fsm::SyncOptions sync;
  static Options compat_defaults();
  static Options fast_defaults();
};

struct Plan {
  std::vector<Action> actions;
  bool requeue = false;
  double requeue_after = 0;  // seconds; 0 = none
  std::string step;          // reconcile step that ended the pass
  api::Status status;        // status after sync
  bool status_changed = false;
};

Plan reconcile(const Observed& obs, const Options& opt, HostPorts* ports, double now);

// helpers shared with tests / the executor
std::string np_key(const api::PaddleJob& job);  // /paddle/<ns>-<name>/np

}  // namespace plan
}  // namespace pdo
