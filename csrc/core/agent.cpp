// SPDX-License-Identifier: Apache-2.0
#include "agent.h"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "builders.h"
#include "log.h"

extern char** environ;

namespace pdo {

using json::Value;

static std::string key_of(const std::string& ns, const std::string& n) { return ns + "/" + n; }

static void mkdirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    mkdir(cur.c_str(), 0755);
  }
}

// "0-3,8,10-11" → cpu ids
static std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    size_t d = tok.find('-');
    if (d == std::string::npos) {
      if (!tok.empty()) out.push_back(atoi(tok.c_str()));
    } else {
      int a = atoi(tok.substr(0, d).c_str()), b = atoi(tok.substr(d + 1).c_str());
      for (int i = a; i <= b; ++i) out.push_back(i);
    }
  }
  return out;
}

Agent::Agent(store::Store* s, AgentOptions o, api::Clock clock, ObjectApi* writer)
    : s_(s), writer_(writer), opt_(std::move(o)), clock_(std::move(clock)) {
  for (int i = 0; i < opt_.node.gpus; ++i) free_gpus_.insert(i);
  mkdirs(opt_.sandbox_root);
  if (opt_.mode == AgentOptions::Exec && !opt_.zygote_cmd.empty()) start_zygote();
}

Agent::~Agent() {
  shutdown();
  stop_zygote();
}

// agent GPU indices -> HIP_VISIBLE_DEVICES values: if the agent itself was
// restricted (HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES), map through it;
// ROCR_VISIBLE_DEVICES is inherited untouched (applied below HIP's list)
static std::string visible_ids(const std::vector<int>& gpus) {
  std::vector<std::string> parent;
  const char* pv = getenv("HIP_VISIBLE_DEVICES");
  if (!pv || !*pv) pv = getenv("CUDA_VISIBLE_DEVICES");
  if (pv && *pv) {
    std::string cur;
    for (const char* q = pv;; ++q) {
      if (*q == ',' || *q == 0) {
        if (!cur.empty()) parent.push_back(cur);
        cur.clear();
        if (!*q) break;
      } else {
        cur += *q;
      }
    }
  }
  std::string ids;
  for (size_t i = 0; i < gpus.size(); ++i) {
    const int g = gpus[i];
    ids += (i ? "," : "") + (g < (int)parent.size() ? parent[g] : std::to_string(g));
  }
  return ids;
}

void Agent::start_zygote() {
  zygote_sock_ = opt_.sandbox_root + "/zygote.sock";
  ::unlink(zygote_sock_.c_str());
  std::vector<std::string> argv = opt_.zygote_cmd;
  argv.push_back("--socket");
  argv.push_back(zygote_sock_);
  // one GPU-warm slot per node GPU (launch/zygote.py); PDO_WARM_SLOTS=0 turns them off
  const char* ws = getenv("PDO_WARM_SLOTS");
  if (opt_.node.gpus > 0 && !(ws && std::string(ws) == "0")) {
    std::vector<int> all;
    for (int i = 0; i < opt_.node.gpus; ++i) all.push_back(i);
    argv.push_back("--warm-devices");
    argv.push_back(visible_ids(all));
  }
  std::vector<char*> av;
  for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  const std::string logp = opt_.sandbox_root + "/zygote.log";
  pid_t pid = fork();
  if (pid == 0) {
    setpgid(0, 0);
    int fd = open(logp.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
      dup2(fd, 1);
      dup2(fd, 2);
      close(fd);
    }
    execvp(av[0], av.data());
    _exit(127);
  }
  if (pid > 0) {
    setpgid(pid, pid);
    zygote_pid_ = pid;
  } else {
    zygote_sock_.clear();
  }
}

void Agent::stop_zygote() {
  if (zygote_pid_ <= 0) return;
  ::kill(zygote_pid_, SIGTERM);
  for (int i = 0; i < 200; ++i) {
    int st;
    if (waitpid(zygote_pid_, &st, WNOHANG) == zygote_pid_) {
      zygote_pid_ = -1;
      break;
    }
    usleep(10000);
  }
  if (zygote_pid_ > 0) {
    ::kill(-zygote_pid_, SIGKILL);
    int st;
    waitpid(zygote_pid_, &st, 0);
    zygote_pid_ = -1;
  }
  ::unlink(zygote_sock_.c_str());
}

bool Agent::zygote_ready() const {
  if (zygote_sock_.empty()) return false;
  struct stat sb;
  return ::stat(zygote_sock_.c_str(), &sb) == 0;
}

size_t Agent::pods() const {
  std::lock_guard<std::mutex> g(mu_);
  return rts_.size();
}

std::string Agent::sandbox_of(const std::string& ns, const std::string& pod) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = rts_.find(key_of(ns, pod));
  return it == rts_.end() ? "" : it->second.sandbox;
}

std::string Agent::alloc_ip() {
  // 127.<block>.<hi>.<lo>, lo in 1..254: every pod its own loopback address
  const int n = ip_seq_++;
  return "127." + std::to_string(opt_.ip_block) + "." + std::to_string((n / 254) % 256) + "." +
         std::to_string(n % 254 + 1);
}

static std::string expand_vars(const std::string& s, const std::map<std::string, std::string>& env) {
  // kubelet $(VAR) expansion; $$(VAR) escapes
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '$' && i + 1 < s.size() && s[i + 1] == '$') {
      out.push_back('$');
      ++i;
      continue;
    }
    if (s[i] == '$' && i + 1 < s.size() && s[i + 1] == '(') {
      size_t close = s.find(')', i + 2);
      if (close != std::string::npos) {
        std::string name = s.substr(i + 2, close - i - 2);
        auto it = env.find(name);
        if (it != env.end()) {
          out += it->second;
          i = close;
          continue;
        }
      }
    }
    out.push_back(s[i]);
  }
  return out;
}

bool Agent::build_env(const Rt& rt, const Value& pod, const Value& c, std::vector<std::string>* env,
                      std::string* err) {
  std::map<std::string, std::string> m;
  std::vector<std::string> order;
  auto set = [&](const std::string& k, const std::string& v) {
    if (!m.count(k)) order.push_back(k);
    m[k] = v;
  };
  const std::string ns = rt.ns;
  for (auto& ef : c.get("envFrom").arr()) {
    const Value& ref = ef.get("configMapRef");
    if (ref.is_null()) continue;
    Value cm;
    if (!s_->try_get("ConfigMap", ns, ref.get("name").str(), &cm)) {
      if (ref.get("optional").as_bool()) continue;
      *err = "configmap \"" + ref.get("name").str() + "\" not found";
      return false;
    }
    const std::string prefix = ef.get("prefix").str();
    for (auto& kv : cm.get("data").obj()) set(prefix + kv.first, kv.second.str());
  }
  for (auto& e : c.get("env").arr()) {
    const std::string name = e.get("name").str();
    if (e.has("value")) {
      set(name, expand_vars(e.get("value").str(), m));
      continue;
    }
    const Value& vf = e.get("valueFrom");
    const Value& fr = vf.get("fieldRef");
    if (!fr.is_null()) {
      const std::string fp = fr.get("fieldPath").str();
      std::string v;
      if (fp == "status.podIP") v = rt.ip;
      else if (fp == "status.hostIP") v = opt_.node.ip;
      else if (fp == "metadata.name") v = rt.name;
      else if (fp == "metadata.namespace") v = rt.ns;
      else if (fp == "metadata.uid") v = rt.uid;
      else if (fp == "spec.nodeName") v = opt_.node.name;
      else if (fp == "spec.serviceAccountName") v = pod.at_path("spec.serviceAccountName").str("default");
      set(name, v);
      continue;
    }
    const Value& ck = vf.get("configMapKeyRef");
    if (!ck.is_null()) {
      Value cm;
      if (!s_->try_get("ConfigMap", ns, ck.get("name").str(), &cm) || !cm.get("data").has(ck.get("key").str())) {
        if (ck.get("optional").as_bool()) continue;
        *err = "configmap key " + ck.get("name").str() + "/" + ck.get("key").str() + " not found";
        return false;
      }
      set(name, cm.get("data").get(ck.get("key").str()).str());
      continue;
    }
    set(name, "");
  }
  // device + sandbox env (the device plugin's job on a real node)
  // PDO_GPU_VISIBILITY=all (node-agent setting): the pod sees every GPU of the
  // node and gets its own ids in PDO_GPU_IDS (bootstrap selects the device),
  // as torchrun-style launches do — RCCL then knows its peers as local devices
  // for xGMI P2P.  Default: HIP_VISIBLE_DEVICES isolation, as a device plugin.
  if (!rt.gpus.empty()) {
    const char* vis = getenv("PDO_GPU_VISIBILITY");
    set(vis && std::string(vis) == "all" ? "PDO_GPU_IDS" : "HIP_VISIBLE_DEVICES", visible_ids(rt.gpus));
  }
  set("PDO_POD_IP", rt.ip);
  set("PDO_NODE_NAME", opt_.node.name);
  set("PDO_SANDBOX", rt.sandbox);
  if (!zygote_sock_.empty() && !m.count("PDO_ZYGOTE")) set("PDO_ZYGOTE", zygote_sock_);
  // inherited agent environment first, pod env overrides
  std::map<std::string, std::string> full;
  for (char** e = environ; e && *e; ++e) {
    std::string kv = *e;
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string k = kv.substr(0, eq);
    if (k == "HIP_VISIBLE_DEVICES" || k == "CUDA_VISIBLE_DEVICES") continue;
    full[k] = kv.substr(eq + 1);
  }
  for (auto& k : order) full[k] = m[k];
  env->clear();
  for (auto& kv : full) env->push_back(kv.first + "=" + kv.second);
  return true;
}

void Agent::start_proc(Rt& rt, const Value& pod, const Value& c, Proc& p, bool is_init) {
  const double now = clock_();
  p.started = true;
  p.started_at = now;
  p.done = false;
  p.reason.clear();
  if (opt_.mode == AgentOptions::Sim) {
    p.running = true;
    return;
  }
  std::vector<std::string> env;
  std::string err;
  if (!build_env(rt, pod, c, &env, &err)) {  // caller checked already; defensive
    p.started = false;
    p.reason = "CreateContainerConfigError";
    return;
  }
  std::map<std::string, std::string> envm;
  for (auto& kv : env) envm[kv.substr(0, kv.find('='))] = kv.substr(kv.find('=') + 1);
  std::vector<std::string> argv;
  for (auto& a : c.get("command").arr()) argv.push_back(expand_vars(a.str(), envm));
  for (auto& a : c.get("args").arr()) argv.push_back(expand_vars(a.str(), envm));
  if (argv.empty()) {
    p.done = true;
    p.running = false;
    p.exit_code = 127;
    p.reason = "RunContainerError";
    p.finished_at = now;
    return;
  }
  std::string cwd = c.get("workingDir").str();
  if (cwd.empty()) cwd = rt.sandbox;
  const std::string logp = rt.sandbox + "/" + c.get("name").str() + ".log";
  std::vector<int> cpus;
  if (!rt.gpus.empty() && rt.gpus[0] < (int)opt_.node.gpu_cpulists.size())
    cpus = parse_cpulist(opt_.node.gpu_cpulists[rt.gpus[0]]);
  // everything the child needs is prepared before fork (async-signal-safe child)
  std::vector<char*> av, ev;
  for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  for (auto& e : env) ev.push_back(const_cast<char*>(e.c_str()));
  ev.push_back(nullptr);
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int cpu : cpus)
    if (cpu >= 0 && cpu < CPU_SETSIZE) CPU_SET(cpu, &set);
  pid_t pid = fork();
  if (pid == 0) {
    setpgid(0, 0);
    int fd = open(logp.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
      dup2(fd, 1);
      dup2(fd, 2);
      close(fd);
    }
    int dn = open("/dev/null", O_RDONLY);
    if (dn >= 0) {
      dup2(dn, 0);
      close(dn);
    }
    if (chdir(cwd.c_str()) != 0) _exit(126);
    if (!cpus.empty()) sched_setaffinity(0, sizeof set, &set);
    execvpe(av[0], av.data(), ev.data());
    _exit(127);
  }
  if (pid < 0) {
    p.done = true;
    p.exit_code = 128;
    p.reason = "StartError";
    return;
  }
  setpgid(pid, pid);
  p.pid = pid;
  p.running = true;
  (void)is_init;
}

void Agent::reap(Rt& rt) {
  auto one = [&](Proc& p) {
    if (!p.running || p.pid <= 0) return;
    int st = 0;
    pid_t r = waitpid(p.pid, &st, WNOHANG);
    if (r == p.pid) {
      p.running = false;
      p.done = true;
      p.finished_at = clock_();
      if (WIFEXITED(st)) {
        p.exit_code = WEXITSTATUS(st);
        p.reason = p.exit_code == 0 ? "Completed" : "Error";
      } else {
        p.exit_code = 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        p.reason = "Error";
      }
      p.pid = -1;
    }
  };
  for (auto& p : rt.init) one(p);
  for (auto& p : rt.main) one(p);
}

bool Agent::all_dead(const Rt& rt) const {
  for (auto& p : rt.init)
    if (p.running) return false;
  for (auto& p : rt.main)
    if (p.running) return false;
  return true;
}

void Agent::terminate(Rt& rt, double now) {
  const bool kill9 = rt.term_sent >= 0 && now - rt.term_sent >= opt_.grace_s;
  if (rt.term_sent < 0) rt.term_sent = now;
  auto sig = [&](Proc& p) {
    if (!p.running) return;
    if (opt_.mode == AgentOptions::Sim) {
      p.running = false;
      p.done = true;
      p.exit_code = 143;
      p.finished_at = now;
      return;
    }
    if (p.pid > 0) ::kill(-p.pid, kill9 ? SIGKILL : SIGTERM);
  };
  for (auto& p : rt.init) sig(p);
  for (auto& p : rt.main) sig(p);
}

void Agent::release(Rt& rt) {
  for (int g : rt.gpus) free_gpus_.insert(g);
  rt.gpus.clear();
}

static Value cstatus(const std::string& name, const std::string& image, bool started, bool running, bool done,
                     int code, int restarts, const std::string& reason, const std::string& waiting,
                     double started_at, double finished_at, bool ready) {
  Value s = Value::object();
  s["name"] = name;
  Value& st = s["state"];
  if (running) {
    st["running"]["startedAt"] = api::rfc3339(started_at);
  } else if (done) {
    st["terminated"]["exitCode"] = code;
    st["terminated"]["reason"] = reason.empty() ? (code == 0 ? "Completed" : "Error") : reason;
    st["terminated"]["startedAt"] = api::rfc3339(started_at);
    st["terminated"]["finishedAt"] = api::rfc3339(finished_at);
  } else {
    st["waiting"]["reason"] = waiting.empty() ? (started ? "ContainerCreating" : "PodInitializing") : waiting;
  }
  s["ready"] = ready;
  s["restartCount"] = restarts;
  s["image"] = image;
  s["started"] = running;
  return s;
}

Value Agent::make_status(const Rt& rt, const Value& pod) const {
  Value st = pod.get("status");
  if (!st.is_object()) st = Value::object();
  const Value& spec = pod.get("spec");
  if (rt.ip_assigned) {
    st["podIP"] = rt.ip;
    Value ips = Value::array();
    Value one = Value::object();
    one["ip"] = rt.ip;
    ips.push_back(one);
    st["podIPs"] = ips;
    st["hostIP"] = opt_.node.ip;
    if (!st.has("startTime")) st["startTime"] = api::rfc3339(rt.t0);
  }
  const auto& ics = spec.get("initContainers").arr();
  Value is = Value::array();
  for (size_t i = 0; i < ics.size() && i < rt.init.size(); ++i) {
    const Proc& p = rt.init[i];
    is.push_back(cstatus(ics[i].get("name").str(), ics[i].get("image").str(), p.started, p.running, p.done,
                         p.exit_code, p.restarts, p.reason, "", p.started_at, p.finished_at,
                         p.done && p.exit_code == 0));
  }
  if (is.size()) st["initContainerStatuses"] = is;
  const auto& cs = spec.get("containers").arr();
  Value ms = Value::array();
  for (size_t i = 0; i < cs.size() && i < rt.main.size(); ++i) {
    const Proc& p = rt.main[i];
    ms.push_back(cstatus(cs[i].get("name").str(), cs[i].get("image").str(), p.started, p.running, p.done,
                         p.exit_code, p.restarts, p.reason, rt.init_idx >= rt.init.size() ? rt.wait_reason : "",
                         p.started_at, p.finished_at, p.running));
  }
  if (ms.size()) st["containerStatuses"] = ms;
  // phase
  const std::string rp = spec.get("restartPolicy").str("Always");
  std::string phase = "Pending";
  bool init_failed = false;
  for (auto& p : rt.init)
    if (p.done && p.exit_code != 0 && rp == "Never") init_failed = true;
  if (init_failed) {
    phase = "Failed";
  } else if (rt.init_idx >= rt.init.size() && !rt.main.empty()) {
    bool any_running = false, all_done = true, all_ok = true;
    for (auto& p : rt.main) {
      if (p.running) any_running = true;
      if (!p.done) all_done = false;
      if (p.done && p.exit_code != 0) all_ok = false;
    }
    if (any_running) phase = "Running";
    else if (all_done && all_ok && rp != "Always") phase = "Succeeded";
    else if (all_done && !all_ok && rp == "Never") phase = "Failed";
    else if (all_done) phase = "Running";  // restarting
  }
  if (rt.terminal) phase = st.get("phase").str(phase);
  st["phase"] = phase;
  Value conds = Value::array();
  auto cond = [&](const char* t, bool v) {
    Value c = Value::object();
    c["type"] = t;
    c["status"] = v ? "True" : "False";
    conds.push_back(c);
  };
  bool ready = phase == "Running";
  for (auto& p : rt.main)
    if (!p.running) ready = false;
  cond("PodScheduled", true);
  cond("Initialized", rt.init_idx >= rt.init.size());
  cond("ContainersReady", ready);
  cond("Ready", ready);
  st["conditions"] = conds;
  return st;
}

bool Agent::step(Rt& rt, const Value& pod, double now) {
  const Value& spec = pod.get("spec");
  const auto& ics = spec.get("initContainers").arr();
  const auto& cs = spec.get("containers").arr();
  const std::string rp = spec.get("restartPolicy").str("Always");
  if (rt.init.size() != ics.size()) rt.init.resize(ics.size());
  if (rt.main.size() != cs.size()) rt.main.resize(cs.size());
  if (!rt.ip_assigned) {
    if (opt_.mode == AgentOptions::Sim && now - rt.t0 < opt_.sim_ip_delay) return false;
    rt.ip_assigned = true;
    return true;
  }
  if (rt.terminal) return false;
  reap(rt);
  // ---- init containers, sequential
  while (rt.init_idx < ics.size()) {
    Proc& p = rt.init[rt.init_idx];
    const Value& c = ics[rt.init_idx];
    const bool coord = c.get("name").as_string() == build::kCoordContainer;
    if (!p.started) {
      start_proc(rt, pod, c, p, true);
      if (opt_.mode == AgentOptions::Sim && !coord) {
        p.running = false;
        p.done = true;
        p.exit_code = 0;
        p.finished_at = now;
      }
      return true;
    }
    if (opt_.mode == AgentOptions::Sim && coord && p.running && rt.coord_released) {
      p.running = false;
      p.done = true;
      p.exit_code = 0;
      p.finished_at = now;
    }
    if (p.running) return false;
    if (p.done && p.exit_code == 0) {
      rt.init_idx++;
      continue;
    }
    if (p.done && rp != "Never") {  // restart failed init container
      p.restarts++;
      p.started = false;
      return true;
    }
    return false;  // init failed with Never → pod Failed (make_status)
  }
  // ---- native start gate (pdo.amd.com/start-gate, released by the controller)
  if (pod.at_path("metadata.annotations").get(api::kAnnotationStartGate).as_string() == api::kGateHold) {
    if (rt.wait_reason != "StartGated") {
      rt.wait_reason = "StartGated";
      return true;
    }
    return false;
  }
  if (rt.wait_reason == "StartGated") rt.wait_reason.clear();
  // ---- main containers
  bool changed = false;
  if (opt_.config_retry_s > 0 && !rt.wait_reason.empty() && now < rt.next_retry) return false;
  for (size_t i = 0; i < cs.size(); ++i) {
    Proc& p = rt.main[i];
    if (p.running) {
      if (opt_.mode == AgentOptions::Sim && opt_.sim_run_s >= 0 && now - p.started_at >= opt_.sim_run_s) {
        p.running = false;
        p.done = true;
        p.exit_code = 0;
        p.finished_at = now;
        changed = true;
      } else {
        continue;
      }
    }
    if (p.started && p.done) {
      const bool restart = rp == "Always" || (rp == "OnFailure" && p.exit_code != 0);
      if (!restart) continue;
      p.restarts++;
      p.started = false;
      changed = true;
    }
    if (!p.started) {
      if (opt_.mode == AgentOptions::Sim && now - rt.t0 < opt_.sim_start_delay) continue;
      std::vector<std::string> env;
      std::string err;
      if (!build_env(rt, pod, cs[i], &env, &err)) {
        if (rt.wait_reason != "CreateContainerConfigError") changed = true;
        rt.wait_reason = "CreateContainerConfigError";
        rt.wait_message = err;
        rt.next_retry = now + opt_.config_retry_s;
        return changed;
      }
      rt.wait_reason.clear();
      start_proc(rt, pod, cs[i], p, false);
      changed = true;
    }
  }
  return changed;
}

int Agent::sync() {
  std::lock_guard<std::mutex> g(mu_);
  const double now = clock_();
  int writes = 0;
  std::set<std::string> seen;
  for (auto& pod : s_->list("Pod")) {
    if (pod.at_path("spec.nodeName").as_string() != opt_.node.name) continue;
    const std::string ns = pod.at_path("metadata.namespace").str();
    const std::string name = pod.at_path("metadata.name").str();
    const std::string key = key_of(ns, name);
    seen.insert(key);
    auto it = rts_.find(key);
    if (it == rts_.end() || it->second.uid != pod.at_path("metadata.uid").as_string()) {
      if (it != rts_.end()) {  // same name, new pod (recreated): drop the stale runtime
        terminate(it->second, now);
        release(it->second);
        rts_.erase(it);
      }
      Rt rt;
      rt.ns = ns;
      rt.name = name;
      rt.uid = pod.at_path("metadata.uid").str();
      rt.t0 = now;
      rt.ip = pod.at_path("spec.hostNetwork").as_bool() ? opt_.node.ip : alloc_ip();
      rt.sandbox = opt_.sandbox_root + "/" + ns + "_" + name + "_" + rt.uid.substr(0, 8);
      mkdirs(rt.sandbox);
      int need = pod_gpu_request(pod);
      for (auto gi = free_gpus_.begin(); gi != free_gpus_.end() && (int)rt.gpus.size() < need;)
        rt.gpus.push_back(*gi), gi = free_gpus_.erase(gi);
      it = rts_.emplace(key, std::move(rt)).first;
    }
    Rt& rt = it->second;
    if (!pod.at_path("metadata.deletionTimestamp").is_null()) {
      reap(rt);
      terminate(rt, now);
      reap(rt);
      if (all_dead(rt)) {
        release(rt);
        try {
          if (writer_) writer_->remove("Pod", ns, name, false);  // grace 0: finalize
          else s_->finalize_delete("Pod", ns, name);
        } catch (const store::ApiError&) {
        }
        rts_.erase(it);
      }
      continue;
    }
    bool changed = false;
    for (int guard = 0; guard < 8 && step(rt, pod, now); ++guard) changed = true;
    reap(rt);
    Value st = make_status(rt, pod);
    const std::string ph = st.get("phase").str();
    if (ph == "Succeeded" || ph == "Failed") {
      rt.terminal = true;
      release(rt);
    }
    if (!(st == pod.get("status"))) {
      Value upd = pod;
      upd["status"] = st;
      upd["metadata"].erase("resourceVersion");
      try {
        if (writer_) writer_->update_status("Pod", upd);
        else s_->update_status("Pod", upd);
        ++writes;
      } catch (const store::ApiError&) {
      }
    }
    (void)changed;
  }
  // pods removed from the store without a graceful delete
  for (auto it = rts_.begin(); it != rts_.end();) {
    if (seen.count(it->first)) {
      ++it;
      continue;
    }
    terminate(it->second, now);
    terminate(it->second, now + opt_.grace_s + 1);
    reap(it->second);
    release(it->second);
    it = rts_.erase(it);
  }
  return writes;
}

bool Agent::exec(const std::string& ns, const std::string& pod, const std::string& container,
                 const std::vector<std::string>& argv, std::string* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = rts_.find(key_of(ns, pod));
  if (it == rts_.end() || argv.empty()) return false;
  Rt& rt = it->second;
  if (opt_.mode == AgentOptions::Sim) {
    if (container == build::kCoordContainer && argv.size() >= 2 && argv[0] == "touch" && argv[1] == "goon")
      rt.coord_released = true;
    return true;
  }
  // run in the pod sandbox (the coordinator loop's cwd) with the pod's env
  pid_t pid = fork();
  if (pid == 0) {
    if (chdir(rt.sandbox.c_str()) != 0) _exit(126);
    std::vector<char*> av;
    for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
    av.push_back(nullptr);
    int dn = open("/dev/null", O_RDWR);
    if (dn >= 0) {
      dup2(dn, 0);
      dup2(dn, 1);
      dup2(dn, 2);
    }
    execvp(av[0], av.data());
    _exit(127);
  }
  if (pid < 0) return false;
  int st = 0;
  const double t0 = clock_();
  while (true) {  // 3 s exec timeout (paddlejob_controller.go:503)
    pid_t r = waitpid(pid, &st, WNOHANG);
    if (r == pid) break;
    if (clock_() - t0 > 3.0) {
      ::kill(pid, SIGKILL);
      waitpid(pid, &st, 0);
      return false;
    }
    usleep(1000);
  }
  if (out) out->clear();
  return WIFEXITED(st) && WEXITSTATUS(st) == 0;
}

bool Agent::kill_pod(const std::string& ns, const std::string& pod, int sig) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = rts_.find(key_of(ns, pod));
  if (it == rts_.end()) return false;
  bool any = false;
  for (auto& p : it->second.main) {
    if (!p.running) continue;
    if (opt_.mode == AgentOptions::Sim) {
      p.running = false;
      p.done = true;
      p.exit_code = 128 + sig;
      p.finished_at = clock_();
    } else if (p.pid > 0) {
      ::kill(-p.pid, sig);
    }
    any = true;
  }
  return any;
}

bool Agent::sim_exit(const std::string& ns, const std::string& pod, int code) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = rts_.find(key_of(ns, pod));
  if (it == rts_.end()) return false;
  for (auto& p : it->second.main) {
    if (!p.running) continue;
    p.running = false;
    p.done = true;
    p.exit_code = code;
    p.reason = code == 0 ? "Completed" : "Error";
    p.finished_at = clock_();
  }
  return true;
}

void Agent::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : rts_) {
    Rt& rt = kv.second;
    for (auto* list : {&rt.init, &rt.main})
      for (auto& p : *list)
        if (p.running && p.pid > 0) ::kill(-p.pid, SIGKILL);
    for (auto* list : {&rt.init, &rt.main})
      for (auto& p : *list)
        if (p.pid > 0) {
          int st;
          waitpid(p.pid, &st, 0);
          p.pid = -1;
          p.running = false;
        }
  }
  rts_.clear();
}

}  // namespace pdo
