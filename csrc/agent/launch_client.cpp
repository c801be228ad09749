// SPDX-License-Identifier: Apache-2.0
// pdo-launch: container entry point of a PaddleJob rank.
//
// Warm path: PDO_ZYGOTE names the per-node zygote's unix socket
// (paddle_operator_amd/launch/zygote.py).  The client sends its argv, full
// environment, cwd and start time (u32 length + JSON) with its fds 0/1/2
// attached (SCM_RIGHTS), then relays SIGTERM/SIGINT/SIGHUP/SIGUSR1/SIGUSR2
// to the forked rank and exits with the rank's status, so the agent still
// supervises one process per container.  If the client itself is SIGKILLed
// the zygote sees EOF and kills the rank's process group.
//
// Cold path (no zygote, or it is unreachable): exec
// `python3 -m paddle_operator_amd.launch <args>` — nothing here touches the
// GPU, so the exec is safe.
#include <errno.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <string>
#include <vector>

extern char** environ;

static volatile sig_atomic_t g_child = 0;

static void relay(int sig) {
  if (g_child > 0) kill(g_child, sig);
}

static std::string json_escape(const char* s) {
  std::string o;
  o.reserve(strlen(s) + 2);
  o += '"';
  for (const unsigned char* p = (const unsigned char*)s; *p; ++p) {
    switch (*p) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (*p < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", *p);
          o += b;
        } else {
          o += (char)*p;
        }
    }
  }
  o += '"';
  return o;
}

static int cold(int argc, char** argv) {
  const char* py = getenv("PDO_PYTHON");
  if (!py || !*py) py = "python3";
  std::vector<char*> av;
  av.push_back((char*)py);
  av.push_back((char*)"-m");
  av.push_back((char*)"paddle_operator_amd.launch");
  for (int i = 1; i < argc; ++i) av.push_back(argv[i]);
  av.push_back(nullptr);
  execvp(py, av.data());
  fprintf(stderr, "pdo-launch: exec %s failed: %s\n", py, strerror(errno));
  return 127;
}

static bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

int main(int argc, char** argv) {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  const double t_start = tv.tv_sec + tv.tv_usec * 1e-6;
  const char* zpath = getenv("PDO_ZYGOTE");
  if (!zpath || !*zpath || getenv("PDO_NO_ZYGOTE")) return cold(argc, argv);

  int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (s < 0 || strlen(zpath) >= sizeof addr.sun_path) return cold(argc, argv);
  strcpy(addr.sun_path, zpath);
  if (connect(s, (sockaddr*)&addr, sizeof addr) != 0) {
    close(s);
    return cold(argc, argv);
  }

  std::string js = "{\"argv\":[";
  for (int i = 1; i < argc; ++i) js += (i > 1 ? "," : "") + json_escape(argv[i]);
  js += "],\"env\":{";
  bool first = true;
  for (char** e = environ; e && *e; ++e) {
    const char* eq = strchr(*e, '=');
    if (!eq) continue;
    std::string k(*e, eq - *e);
    js += (first ? "" : ",") + json_escape(k.c_str()) + ":" + json_escape(eq + 1);
    first = false;
  }
  char cwd[4096];
  if (!getcwd(cwd, sizeof cwd)) strcpy(cwd, "/");
  char ts[64];
  snprintf(ts, sizeof ts, "%.6f", t_start);
  js += "},\"cwd\":" + json_escape(cwd) + ",\"t_start\":" + ts + "}";

  // header + fds in one sendmsg, body after
  uint32_t n = (uint32_t)js.size();
  int fds[3] = {0, 1, 2};
  char cbuf[CMSG_SPACE(sizeof fds)];
  memset(cbuf, 0, sizeof cbuf);
  iovec iov{&n, sizeof n};
  msghdr mh{};
  mh.msg_iov = &iov;
  mh.msg_iovlen = 1;
  mh.msg_control = cbuf;
  mh.msg_controllen = sizeof cbuf;
  cmsghdr* cm = CMSG_FIRSTHDR(&mh);
  cm->cmsg_level = SOL_SOCKET;
  cm->cmsg_type = SCM_RIGHTS;
  cm->cmsg_len = CMSG_LEN(sizeof fds);
  memcpy(CMSG_DATA(cm), fds, sizeof fds);
  if (sendmsg(s, &mh, MSG_NOSIGNAL) != (ssize_t)sizeof n || !send_all(s, js.data(), js.size())) {
    close(s);
    return cold(argc, argv);
  }

  struct sigaction sa{};
  sa.sa_handler = relay;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGTERM, SIGINT, SIGHUP, SIGUSR1, SIGUSR2}) sigaction(sig, &sa, nullptr);

  std::string buf;
  char tmp[256];
  for (;;) {
    ssize_t r = recv(s, tmp, sizeof tmp, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    buf.append(tmp, (size_t)r);
    size_t nl;
    while ((nl = buf.find('\n')) != std::string::npos) {
      std::string line = buf.substr(0, nl);
      buf.erase(0, nl + 1);
      if (line.rfind("PID ", 0) == 0) {
        g_child = atoi(line.c_str() + 4);
      } else if (line.rfind("EXIT ", 0) == 0) {
        close(s);
        return atoi(line.c_str() + 5);
      }
    }
  }
  fprintf(stderr, "pdo-launch: zygote connection lost\n");
  close(s);
  return 125;
}
