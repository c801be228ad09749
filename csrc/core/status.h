// SPDX-License-Identifier: Apache-2.0
// Status aggregation + phase/mode state machine of a PaddleJob.
//
// Reference semantics: controllers/paddlejob_controller.go:335-381
// (syncCurrentStatus) and paddlejob_helper.go:76-199 (predicates,
// getPaddleJobPhase, start/completion time, mode).  Two deliberate, documented
// differences:
//  * D-1 fixed in both modes: roles are evaluated in the fixed order
//    ps → worker → heter with priority Failed > Starting > Pending across ALL
//    roles (the reference iterates a Go map and returns on the first hit).
//  * D-2 (one-pass phase lag: phase derived from the PREVIOUS pass's counts)
//    is reproduced only when `compat_phase_lag` is set.
#pragma once

#include <string>
#include <vector>

#include "api.h"

namespace pdo {
namespace fsm {

using json::Value;

bool pod_really_running(const Value& pod);   // isPodRealRuning
bool coord_running(const Value& pod);        // isCoordContainerRunning
bool all_coord_running(const std::vector<Value>& pods);
bool all_pods_created(const api::PaddleJob& job);
bool all_pods_ready(const api::PaddleJob& job, const std::vector<Value>& pods);  // PodIP != ""

std::string derive_phase(const api::PaddleJob& job);  // from job.status counts
std::string derive_mode(const api::Spec& spec);

struct SyncOptions {
  bool compat_phase_lag = false;  // reproduce D-2
  bool count_unknown = true;      // fill ResourceStatus.unknown (never set by the reference)
  bool set_observed_generation = true;  // fix D-13 (observedGeneration always 0 in the reference)
};

// new status of `job` given its child pods (pods of this job only)
api::Status sync_status(const api::PaddleJob& job, const std::vector<Value>& pods, double now,
                        const SyncOptions& opt);

}  // namespace fsm
}  // namespace pdo
