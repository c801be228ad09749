// SPDX-License-Identifier: Apache-2.0
// pdo-agent: standalone kubelet-lite joining a pdo-manager (local backend)
// from another host / container:
//   pdo-agent --server http://manager:8082 --node gpu-node-1 --gpus 8
// The manager must list the node (pdo-manager --remote-node gpu-node-1=8).
// Pods are mirrored from the manager's REST API (list+watch informer) and
// pod status / final deletes are written back through the same API.
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>

#include "agent.h"
#include "k8s.h"
#include "log.h"

static std::atomic<bool> g_stop{false};
static void on_sig(int) { g_stop = true; }

int main(int argc, char** argv) {
  std::string server = "http://127.0.0.1:8082", node = "local", sandbox = "/tmp/pdo-agent", ip = "127.0.0.1";
  int gpus = 0, block = 2;
  std::string mode = "exec";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--server") server = next();
    else if (a == "--node") node = next();
    else if (a == "--gpus") gpus = atoi(next().c_str());
    else if (a == "--sandbox-root") sandbox = next();
    else if (a == "--node-ip") ip = next();
    else if (a == "--ip-block") block = atoi(next().c_str());
    else if (a == "--mode") mode = next();
    else if (a == "-h" || a == "--help") {
      printf("pdo-agent --server URL --node NAME --gpus N [--sandbox-root DIR] [--node-ip IP] [--mode exec|sim]\n");
      return 0;
    }
  }
  signal(SIGTERM, on_sig);
  signal(SIGINT, on_sig);
  signal(SIGPIPE, SIG_IGN);
  pdo::k8s::Config cfg;
  cfg.server = server;
  pdo::k8s::RestApi api(cfg);
  pdo::store::Store cache;
  pdo::k8s::Informer pods(&api, &cache, "Pod", "");
  pdo::k8s::Informer cms(&api, &cache, "ConfigMap", "");
  pods.start();
  cms.start();
  pdo::AgentOptions ao;
  ao.mode = mode == "sim" ? pdo::AgentOptions::Sim : pdo::AgentOptions::Exec;
  ao.node.name = node;
  ao.node.ip = ip;
  ao.node.gpus = gpus;
  ao.sandbox_root = sandbox + "/" + node;
  ao.ip_block = block;
  pdo::Agent agent(&cache, ao, pdo::api::wall_clock, &api);
  pdo::log::info("pdo-agent", "started", {{"server", server}, {"node", node}, {"gpus", std::to_string(gpus)}});
  while (!g_stop) {
    cache.drain();
    agent.sync();
    cache.wait_events(0.05);
  }
  agent.shutdown();
  pods.stop();
  cms.stop();
  return 0;
}
