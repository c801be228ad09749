// SPDX-License-Identifier: Apache-2.0
#pragma once
#include <string>

namespace pdo {
std::string b64encode(const std::string& in);
bool b64decode(const std::string& in, std::string* out);
}  // namespace pdo
