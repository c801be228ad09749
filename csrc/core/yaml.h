// SPDX-License-Identifier: Apache-2.0
// Minimal YAML → JSON DOM reader for kubeconfig files and Kubernetes
// manifests (block mappings/sequences, plain/quoted scalars, literal `|` and
// folded `>` blocks, simple flow collections, comments, `---` documents).
// Not supported: anchors/aliases, tags, complex keys.
#pragma once

#include <string>
#include <vector>

#include "json.h"

namespace pdo {
namespace yaml {

std::vector<json::Value> parse_all(const std::string& text);  // one Value per document
json::Value parse(const std::string& text);                     // first document

}  // namespace yaml
}  // namespace pdo
