// SPDX-License-Identifier: Apache-2.0
// pdo-agent: "kubelet-lite" for the local backend.
//
// Runs the pods bound to one node.  Exec mode starts real processes (one
// process group per container, stdout/stderr → <sandbox>/<container>.log),
// Sim mode advances a scripted timeline (for control-plane tests and
// multi-node simulation without hardware).  Both report the pod status
// fields the reference controller reads (phase, podIP, init/container
// statuses with state.running / ready: paddlejob_helper.go:134-173).
//
// MI355X-native parts (SURVEY §2.2 "pdo-agent"): amd.com/gpu requests are
// satisfied by exclusive GPU indices exported as HIP_VISIBLE_DEVICES (one
// rank per MI355X), the process is pinned to the GPU's NUMA-local CPUs
// (sysfs local_cpulist), every pod gets its own loopback address
// 127.<a>.<b>.<c> (IPv4, own port space: several PaddleJob pods can all
// listen on :2379 on one node), and envFrom/fieldRef/$(VAR) are resolved as
// kubelet does.  The reference's coordinator init container
// (`sh -c 'until [ -f goon ]…'`) runs for real and `exec` creates the file.
#pragma once

#include <sys/types.h>

#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "objectapi.h"
#include "scheduler.h"
#include "store.h"

namespace pdo {

struct AgentOptions {
  enum Mode { Exec, Sim } mode = Sim;
  NodeInfo node;
  std::string sandbox_root = "/tmp/pdo-agent";
  double config_retry_s = 0;  // >0: retry CreateContainerConfigError only every N s (kubelet backoff, compat)
  double grace_s = 2.0;       // SIGTERM → SIGKILL
  int ip_block = 1;           // second octet of pod IPs (127.<block>.x.y)
  // sim timeline
  double sim_ip_delay = 0.0;
  double sim_start_delay = 0.0;
  double sim_run_s = -1;  // <0: run until told otherwise
  // warm launcher: argv of a per-node zygote (launch/zygote.py) started with
  // the agent; its socket is exported to pods as PDO_ZYGOTE (Exec mode)
  std::vector<std::string> zygote_cmd;
};

class Agent {
 public:
  // `s`: where pods are read (the API server itself, or an informer cache);
  // `writer`: where status / final deletes go (nullptr → `s`)
  Agent(store::Store* s, AgentOptions o, api::Clock clock = api::wall_clock, ObjectApi* writer = nullptr);
  ~Agent();
  Agent(const Agent&) = delete;
  Agent& operator=(const Agent&) = delete;

  // advance every pod of this node one step; returns #status updates written
  int sync();
  // run argv in `container` of the pod (kubectl exec); true on exit 0
  bool exec(const std::string& ns, const std::string& pod, const std::string& container,
            const std::vector<std::string>& argv, std::string* out = nullptr);
  // fault injection: signal the main container process groups (Exec) /
  // terminate main containers with `code` (Sim)
  bool kill_pod(const std::string& ns, const std::string& pod, int sig);
  bool sim_exit(const std::string& ns, const std::string& pod, int code);
  void shutdown();
  size_t pods() const;
  const AgentOptions& options() const { return opt_; }
  std::string sandbox_of(const std::string& ns, const std::string& pod) const;
  // zygote socket path ("" if none) and whether it is accepting
  const std::string& zygote_socket() const { return zygote_sock_; }
  bool zygote_ready() const;

 private:
  struct Proc {
    pid_t pid = -1;
    bool started = false, running = false, done = false;
    int exit_code = 0;
    int restarts = 0;
    double started_at = 0, finished_at = 0;
    std::string reason;
  };
  struct Rt {
    std::string ns, name, uid, ip, sandbox;
    std::vector<int> gpus;
    std::vector<Proc> init, main;
    size_t init_idx = 0;
    double t0 = 0;
    bool ip_assigned = false;
    bool coord_released = false;  // sim coord emulation
    std::string wait_reason, wait_message;
    double next_retry = 0;
    double term_sent = -1;
    bool terminal = false;
  };

  void start_proc(Rt& rt, const json::Value& pod, const json::Value& container, Proc& p, bool is_init);
  bool build_env(const Rt& rt, const json::Value& pod, const json::Value& container,
                 std::vector<std::string>* env, std::string* err);
  void reap(Rt& rt);
  bool step(Rt& rt, const json::Value& pod, double now);
  json::Value make_status(const Rt& rt, const json::Value& pod) const;
  void terminate(Rt& rt, double now);
  bool all_dead(const Rt& rt) const;
  void release(Rt& rt);
  std::string alloc_ip();

  store::Store* s_;
  ObjectApi* writer_ = nullptr;
  AgentOptions opt_;
  api::Clock clock_;
  mutable std::mutex mu_;
  std::map<std::string, Rt> rts_;  // ns/name
  std::set<int> free_gpus_;
  int ip_seq_ = 0;
  pid_t zygote_pid_ = -1;
  std::string zygote_sock_;
  void start_zygote();
  void stop_zygote();
};

}  // namespace pdo
