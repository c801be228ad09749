// SPDX-License-Identifier: Apache-2.0
#include "log.h"

#include <sys/time.h>

#include <cstdio>
#include <ctime>
#include <mutex>

#include "json.h"

namespace pdo {
namespace log {

static Config g_cfg;
static std::mutex g_mu;

void configure(const Config& c) { g_cfg = c; }
Config& config() { return g_cfg; }

bool parse_level(const std::string& s, Level* out) {
  if (s == "debug") *out = Debug;
  else if (s == "info") *out = Info;
  else if (s == "warn") *out = Warn;
  else if (s == "error") *out = Error;
  else {
    char* end = nullptr;
    long v = strtol(s.c_str(), &end, 10);
    if (!end || *end) return false;
    *out = (Level)(v > 0 ? -1 : 0);  // zap: positive integers enable debug verbosity
  }
  return true;
}

static const char* lname(Level l) {
  switch (l) {
    case Debug: return "debug";
    case Info: return "info";
    case Warn: return "warn";
    case Error: return "error";
  }
  return "info";
}

void write(Level lv, const std::string& logger, const std::string& msg, const KV& kv) {
  if (lv < g_cfg.level) return;
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  std::lock_guard<std::mutex> g(g_mu);
  if (g_cfg.json) {
    json::Value o = json::Value::object();
    o["level"] = lname(lv);
    o["ts"] = tv.tv_sec + tv.tv_usec * 1e-6;
    o["logger"] = logger;
    o["msg"] = msg;
    for (auto& p : kv) o[p.first] = p.second;
    fprintf(stderr, "%s\n", o.dump().c_str());
  } else {
    struct tm tmv;
    gmtime_r(&tv.tv_sec, &tmv);
    char ts[40];
    strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%S", &tmv);
    std::string line = std::string(ts) + "." + std::to_string(tv.tv_usec / 1000) + "Z\t" + lname(lv) + "\t" +
                       logger + "\t" + msg;
    if (!kv.empty()) {
      json::Value o = json::Value::object();
      for (auto& p : kv) o[p.first] = p.second;
      line += "\t" + o.dump();
    }
    fprintf(stderr, "%s\n", line.c_str());
  }
}

}  // namespace log
}  // namespace pdo
