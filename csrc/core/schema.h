// SPDX-License-Identifier: Apache-2.0
// Structural-schema admission for PaddleJob: the apiserver behaviour the
// reference gets from its CRD's embedded PodTemplateSpec schema
// (deploy/v1/crd.yaml:59-3146) — unknown fields pruned on write, required
// fields and types checked (422 Invalid).  The schema is the CRD's own
// openAPIV3Schema (paddle_operator_amd/api/crd.py), compiled in from
// crd_schema.inc; `python -m paddle_operator_amd.deploy` regenerates both.
#pragma once

#include <string>
#include <vector>

#include "json.h"

namespace pdo {
namespace schema {

using json::Value;

// drop object fields the schema does not declare (unless the node has
// x-kubernetes-preserve-unknown-fields); the root's `metadata` is kept
void prune(Value& v, const Value& s, bool root = true);
// "<path>: <message>" for type mismatches and missing required fields
void check(const Value& v, const Value& s, const std::string& path, std::vector<std::string>* errs);

const Value& paddlejob_schema();
// prune + check a PaddleJob about to be written; throws store::ApiError(Invalid)
void admit_paddlejob(Value& obj);

}  // namespace schema
}  // namespace pdo
