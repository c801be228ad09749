// SPDX-License-Identifier: Apache-2.0
// Structured logging (zap-compatible flags: --zap-devel, --zap-log-level,
// --zap-encoder=json|console; reference main.go:79-85).
#pragma once

#include <string>
#include <utility>
#include <vector>

namespace pdo {
namespace log {

enum Level { Debug = -1, Info = 0, Warn = 1, Error = 2 };

struct Config {
  Level level = Info;
  bool json = false;    // --zap-encoder=json
  bool devel = true;    // reference default Development=true
};

void configure(const Config& c);
Config& config();
bool parse_level(const std::string& s, Level* out);

using KV = std::vector<std::pair<std::string, std::string>>;
void write(Level lv, const std::string& logger, const std::string& msg, const KV& kv = {});
inline void info(const std::string& logger, const std::string& msg, const KV& kv = {}) { write(Info, logger, msg, kv); }
inline void error(const std::string& logger, const std::string& msg, const KV& kv = {}) { write(Error, logger, msg, kv); }
inline void debug(const std::string& logger, const std::string& msg, const KV& kv = {}) { write(Debug, logger, msg, kv); }

}  // namespace log
}  // namespace pdo
