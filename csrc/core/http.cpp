// SPDX-License-Identifier: Apache-2.0
#include "http.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <fcntl.h>
#include <poll.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstring>
#include <deque>
#include <random>
#include <sstream>

#include "base64.h"
#include "json.h"

#ifdef PDO_WITH_TLS
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#endif

namespace pdo {
namespace http {

static std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::string url_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size()) {
      out.push_back((char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
      i += 2;
    } else if (s[i] == '+') {
      out.push_back(' ');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

std::string Request::param(const std::string& k, const std::string& def) const {
  size_t pos = 0;
  while (pos <= query.size()) {
    size_t amp = query.find('&', pos);
    std::string kv = query.substr(pos, amp == std::string::npos ? std::string::npos : amp - pos);
    size_t eq = kv.find('=');
    std::string key = url_decode(kv.substr(0, eq));
    if (key == k) return eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1));
    if (amp == std::string::npos) break;
    pos = amp + 1;
  }
  return def;
}

std::vector<std::string> Request::params(const std::string& k) const {
  std::vector<std::string> out;
  size_t pos = 0;
  while (pos <= query.size()) {
    size_t amp = query.find('&', pos);
    std::string kv = query.substr(pos, amp == std::string::npos ? std::string::npos : amp - pos);
    size_t eq = kv.find('=');
    if (url_decode(kv.substr(0, eq)) == k) out.push_back(eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1)));
    if (amp == std::string::npos) break;
    pos = amp + 1;
  }
  return out;
}

std::string url_encode(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string out;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out.push_back((char)c);
    } else {
      out.push_back('%');
      out.push_back(hex[c >> 4]);
      out.push_back(hex[c & 15]);
    }
  }
  return out;
}

static const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 101: return "Switching Protocols";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 422: return "Unprocessable Entity";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
  }
  return "Status";
}

static bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w <= 0) {
      if (w < 0 && errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

// ------------------------------------------------------------------ server
Server::~Server() { stop(); }

void Server::route(const std::string& method, const std::string& path, Handler h) {
  Route r;
  r.method = method;
  r.prefix = !path.empty() && path.back() == '*';
  r.path = r.prefix ? path.substr(0, path.size() - 1) : path;
  r.h = std::move(h);
  routes_.push_back(std::move(r));
}

const Handler* Server::match(const std::string& method, const std::string& path) const {
  const Route* best = nullptr;
  for (auto& r : routes_) {
    if (r.method != "*" && r.method != method) continue;
    if (r.prefix ? path.compare(0, r.path.size(), r.path) == 0 : path == r.path) {
      if (!best || (!r.prefix && best->prefix) || (r.prefix && best->prefix && r.path.size() > best->path.size()))
        best = &r;
    }
  }
  return best ? &best->h : nullptr;
}

int Server::listen(const std::string& addr) {
  std::string host = "0.0.0.0";
  std::string port_s = addr;
  size_t c = addr.rfind(':');
  if (c != std::string::npos) {
    if (c > 0) host = addr.substr(0, c);
    port_s = addr.substr(c + 1);
  }
  if (addr == "0" || port_s.empty()) port_s = "0";
  fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd_ < 0) return -1;
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)atoi(port_s.c_str()));
  if (inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) sa.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(fd_, (sockaddr*)&sa, sizeof sa) < 0 || ::listen(fd_, 128) < 0) {
    ::close(fd_);
    fd_ = -1;
    return -1;
  }
  socklen_t len = sizeof sa;
  getsockname(fd_, (sockaddr*)&sa, &len);
  port_ = ntohs(sa.sin_port);
  return port_;
}

void Server::start() {
  if (fd_ < 0 || running_) return;
  running_ = true;
  acceptor_ = std::thread([this] { accept_loop(); });
}

void Server::stop() {
  if (!running_.exchange(false)) {
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
    return;
  }
  // wake the acceptor (shutdown makes its accept4 fail), join it, THEN close:
  // closing first would let the acceptor read fd_ concurrently (TSan) and call
  // accept4 on a descriptor number the process may already have reused
  ::shutdown(fd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  ::close(fd_);
  fd_ = -1;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int cfd : conn_fds_) ::shutdown(cfd, SHUT_RDWR);
  }
  // connection threads are detached; wait (bounded) for them to leave
  for (int i = 0; i < 500 && active_.load() > 0; ++i) usleep(2000);
}

void Server::accept_loop() {
  const int lfd = fd_;  // fixed for the acceptor's lifetime (stop() closes it after the join)
  while (running_) {
    sockaddr_in sa{};
    socklen_t len = sizeof sa;
    int cfd = ::accept4(lfd, (sockaddr*)&sa, &len, SOCK_CLOEXEC);
    if (cfd < 0) {
      if (!running_) break;
      if (errno == EINTR) continue;
      usleep(1000);
      continue;
    }
    int one = 1;
    setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    std::lock_guard<std::mutex> g(conn_mu_);
    conn_fds_.push_back(cfd);
    active_++;
    std::thread([this, cfd] { serve(cfd); }).detach();
  }
}

namespace {
class ChunkWriter : public StreamWriter {
 public:
  explicit ChunkWriter(int fd) : fd_(fd) {}
  bool write(const std::string& chunk) override {
    if (closed_) return false;
    if (chunk.empty()) return true;
    char hdr[32];
    int n = snprintf(hdr, sizeof hdr, "%zx\r\n", chunk.size());
    if (!send_all(fd_, hdr, n) || !send_all(fd_, chunk.data(), chunk.size()) || !send_all(fd_, "\r\n", 2)) {
      closed_ = true;
      return false;
    }
    return true;
  }
  bool closed() const override {
    if (closed_) return true;
    char b;
    ssize_t r = ::recv(fd_, &b, 1, MSG_PEEK | MSG_DONTWAIT);
    return r == 0;
  }
  void finish() {
    if (!closed_) send_all(fd_, "0\r\n\r\n", 5);
  }

 private:
  int fd_;
  mutable bool closed_ = false;
};
}  // namespace

void Server::serve(int fd) {
  std::string buf;
  char tmp[16384];
  bool keep = true;
  while (keep && running_) {
    size_t hdr_end;
    while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
      ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r <= 0) goto done;
      buf.append(tmp, (size_t)r);
      if (buf.size() > (1u << 20)) goto done;
    }
    {
      Request req;
      std::istringstream hs(buf.substr(0, hdr_end));
      std::string line;
      std::getline(hs, line);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      std::istringstream rl(line);
      std::string target, ver;
      rl >> req.method >> target >> ver;
      size_t q = target.find('?');
      req.path = q == std::string::npos ? target : target.substr(0, q);
      req.query = q == std::string::npos ? "" : target.substr(q + 1);
      while (std::getline(hs, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        size_t colon = line.find(':');
        if (colon == std::string::npos) continue;
        std::string v = line.substr(colon + 1);
        v.erase(0, v.find_first_not_of(' '));
        req.headers[lower(line.substr(0, colon))] = v;
      }
      size_t clen = req.headers.count("content-length") ? (size_t)atol(req.headers["content-length"].c_str()) : 0;
      buf.erase(0, hdr_end + 4);
      while (buf.size() < clen) {
        ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
        if (r <= 0) goto done;
        buf.append(tmp, (size_t)r);
      }
      req.body = buf.substr(0, clen);
      buf.erase(0, clen);
      if (lower(req.headers["connection"]) == "close" || ver == "HTTP/1.0") keep = false;

      Response resp;
      const Handler* h = match(req.method, req.path);
      if (!h) {
        resp.status = 404;
        resp.body = "{\"kind\":\"Status\",\"status\":\"Failure\",\"reason\":\"NotFound\",\"code\":404}";
      } else {
        try {
          resp = (*h)(req);
        } catch (const std::exception& e) {
          resp.status = 500;
          resp.content_type = "text/plain";
          resp.body = e.what();
        }
      }
      if (resp.upgrade) {
        std::string head = "HTTP/1.1 101 Switching Protocols\r\n";
        for (auto& kv : resp.headers) head += kv.first + ": " + kv.second + "\r\n";
        head += "\r\n";
        if (send_all(fd, head.data(), head.size())) resp.upgrade(fd);
        goto done;
      }
      std::string head = "HTTP/1.1 " + std::to_string(resp.status) + " " + reason(resp.status) + "\r\n";
      head += "Content-Type: " + resp.content_type + "\r\n";
      for (auto& kv : resp.headers) head += kv.first + ": " + kv.second + "\r\n";
      if (resp.stream) {
        head += "Transfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
        if (!send_all(fd, head.data(), head.size())) goto done;
        ChunkWriter w(fd);
        resp.stream(w);
        w.finish();
        goto done;
      }
      head += "Content-Length: " + std::to_string(resp.body.size()) + "\r\n";
      head += keep ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
      if (!send_all(fd, head.data(), head.size()) || !send_all(fd, resp.body.data(), resp.body.size())) goto done;
    }
  }
done:
  ::close(fd);
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    conn_fds_.erase(std::remove(conn_fds_.begin(), conn_fds_.end(), fd), conn_fds_.end());
  }
  active_--;
}

// ------------------------------------------------------------------ client
bool parse_url(const std::string& url, std::string* scheme, std::string* host, int* port, std::string* path) {
  size_t p = url.find("://");
  std::string rest = url;
  *scheme = "http";
  if (p != std::string::npos) {
    *scheme = url.substr(0, p);
    rest = url.substr(p + 3);
  }
  size_t slash = rest.find('/');
  std::string hp = rest.substr(0, slash);
  *path = slash == std::string::npos ? "/" : rest.substr(slash);
  size_t colon = hp.rfind(':');
  if (colon != std::string::npos && hp.find(']') == std::string::npos) {
    *host = hp.substr(0, colon);
    *port = atoi(hp.substr(colon + 1).c_str());
  } else {
    *host = hp;
    *port = *scheme == "https" ? 443 : 80;
  }
  return !host->empty();
}

namespace {

#ifdef PDO_WITH_TLS
// PEM text → certificates / key through memory BIOs: kubeconfig *-data
// material is never written to a file
bool load_pem_ca(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), (int)pem.size());
  if (!bio) return false;
  X509_STORE* store = SSL_CTX_get_cert_store(ctx);
  int n = 0;
  while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
    if (X509_STORE_add_cert(store, x) == 1) ++n;
    X509_free(x);
  }
  ERR_clear_error();  // the read loop ends on a "no start line" error
  BIO_free(bio);
  return n > 0;
}

bool load_pem_cert(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), (int)pem.size());
  if (!bio) return false;
  X509* leaf = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
  bool ok = leaf && SSL_CTX_use_certificate(ctx, leaf) == 1;
  while (ok) {  // intermediates after the leaf
    X509* extra = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
    if (!extra) break;
    if (SSL_CTX_add_extra_chain_cert(ctx, extra) != 1) {  // takes ownership on success
      X509_free(extra);
      ok = false;
    }
  }
  ERR_clear_error();
  if (leaf) X509_free(leaf);
  BIO_free(bio);
  return ok;
}

bool load_pem_key(SSL_CTX* ctx, const std::string& pem) {
  BIO* bio = BIO_new_mem_buf(pem.data(), (int)pem.size());
  if (!bio) return false;
  EVP_PKEY* k = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  const bool ok = k && SSL_CTX_use_PrivateKey(ctx, k) == 1;
  if (k) EVP_PKEY_free(k);
  BIO_free(bio);
  return ok;
}
#endif

std::string tls_identity(const ClientOptions& o) {
  return o.ca_file + '\n' + o.cert_file + '\n' + o.key_file + '\n' + o.ca_pem + '\n' + o.cert_pem + '\n' + o.key_pem +
         (o.insecure_skip_verify ? "\ninsecure" : "\nverify");
}

#ifdef PDO_WITH_TLS
// one SSL_CTX per distinct trust/identity configuration, shared by every
// connection that uses it (handshakes reuse the loaded chain and key)
SSL_CTX* tls_context(const ClientOptions& opt, std::string* err) {
  static std::mutex mu;
  static std::map<std::string, SSL_CTX*> cache;  // process lifetime
  const std::string key = tls_identity(opt);
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) {
    *err = "SSL_CTX_new failed";
    return nullptr;
  }
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  bool ok = true;
  if (!opt.ca_pem.empty()) {
    ok = load_pem_ca(ctx, opt.ca_pem);
    if (!ok) *err = "cannot load the CA certificate (PEM data)";
  } else if (!opt.ca_file.empty()) {
    ok = SSL_CTX_load_verify_locations(ctx, opt.ca_file.c_str(), nullptr) == 1;
    if (!ok) *err = "cannot load the CA certificate " + opt.ca_file;
  } else {
    SSL_CTX_set_default_verify_paths(ctx);
  }
  const bool has_cert = !opt.cert_pem.empty() || !opt.cert_file.empty();
  const bool has_key = !opt.key_pem.empty() || !opt.key_file.empty();
  if (ok && has_cert) {
    ok = !opt.cert_pem.empty() ? load_pem_cert(ctx, opt.cert_pem)
                               : SSL_CTX_use_certificate_chain_file(ctx, opt.cert_file.c_str()) == 1;
    if (!ok) *err = "cannot load the client certificate";
  }
  if (ok && has_key) {
    ok = !opt.key_pem.empty() ? load_pem_key(ctx, opt.key_pem)
                              : SSL_CTX_use_PrivateKey_file(ctx, opt.key_file.c_str(), SSL_FILETYPE_PEM) == 1;
    if (!ok) *err = "cannot load the client key";
  }
  if (ok && (has_cert || has_key)) {
    ok = has_cert && has_key && SSL_CTX_check_private_key(ctx) == 1;
    if (!ok) *err = "client certificate and key do not match (or one is missing)";
  }
  if (!ok) {
    ERR_clear_error();
    SSL_CTX_free(ctx);
    return nullptr;
  }
  SSL_CTX_set_verify(ctx, opt.insecure_skip_verify ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
  cache[key] = ctx;
  return ctx;
}
#endif

struct Conn {
  int fd = -1;
  std::string pool_key;
#ifdef PDO_WITH_TLS
  SSL* ssl = nullptr;
#endif
  Conn() = default;
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;
  ~Conn() { close(); }
  void close() {
#ifdef PDO_WITH_TLS
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
      ssl = nullptr;
    }
#endif
    if (fd >= 0) {
      ::close(fd);
      fd = -1;
    }
  }
  ssize_t rd(char* b, size_t n) {
#ifdef PDO_WITH_TLS
    if (ssl) return SSL_read(ssl, b, (int)n);
#endif
    return ::recv(fd, b, n, 0);
  }
  bool wr(const std::string& s) {
#ifdef PDO_WITH_TLS
    if (ssl) return SSL_write(ssl, s.data(), (int)s.size()) == (int)s.size();
#endif
    return send_all(fd, s.data(), s.size());
  }
  void set_timeout(double t) {
    timeval tv;
    tv.tv_sec = (long)t;
    tv.tv_usec = (long)((t - (long)t) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  }
  // an idle pooled connection is reusable only if nothing is readable on it:
  // readable = the server closed it (EOF) or sent stray bytes
  bool idle_ok() const {
    if (fd < 0) return false;
#ifdef PDO_WITH_TLS
    if (ssl && SSL_pending(ssl) > 0) return false;
#endif
    pollfd p{fd, POLLIN, 0};
    return ::poll(&p, 1, 0) == 0;
  }
};

// idle keep-alive connections per (server, TLS identity); bounded per key
std::mutex g_pool_mu;
std::map<std::string, std::deque<std::unique_ptr<Conn>>> g_pool;
constexpr size_t kPoolPerKey = 8;

std::unique_ptr<Conn> pool_take(const std::string& key) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto it = g_pool.find(key);
  if (it == g_pool.end()) return nullptr;
  while (!it->second.empty()) {
    std::unique_ptr<Conn> c = std::move(it->second.back());
    it->second.pop_back();
    if (c->idle_ok()) return c;
  }
  return nullptr;
}

void pool_put(std::unique_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto& q = g_pool[c->pool_key];
  if (q.size() < kPoolPerKey) q.push_back(std::move(c));
}

bool is_ip_literal(const std::string& host) {
  unsigned char buf[sizeof(in6_addr)];
  return inet_pton(AF_INET, host.c_str(), buf) == 1 || inet_pton(AF_INET6, host.c_str(), buf) == 1;
}

// connect with a deadline (non-blocking connect + poll), close-on-exec socket
int connect_timeout(const addrinfo* a, double timeout_s) {
  int fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, a->ai_protocol);
  if (fd < 0) return -1;
  int rc = ::connect(fd, a->ai_addr, a->ai_addrlen);
  if (rc != 0 && errno == EINPROGRESS) {
    pollfd p{fd, POLLOUT, 0};
    rc = ::poll(&p, 1, (int)(timeout_s * 1000)) == 1 ? 0 : -1;
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    if (rc == 0 && (getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) != 0 || soerr != 0)) rc = -1;
  }
  if (rc != 0) {
    ::close(fd);
    return -1;
  }
  fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) & ~O_NONBLOCK);
  return fd;
}

bool dial(Conn& c, const std::string& scheme, const std::string& host, int port, const ClientOptions& opt,
          std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    *err = "resolve " + host + " failed";
    return false;
  }
  for (addrinfo* a = res; a && c.fd < 0; a = a->ai_next) c.fd = connect_timeout(a, opt.timeout_s);
  freeaddrinfo(res);
  if (c.fd < 0) {
    *err = "connect " + host + ":" + std::to_string(port) + " failed";
    return false;
  }
  c.set_timeout(opt.timeout_s);
  int one = 1;
  setsockopt(c.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  if (scheme == "https") {
#ifdef PDO_WITH_TLS
    SSL_CTX* ctx = tls_context(opt, err);
    if (!ctx) return false;
    c.ssl = SSL_new(ctx);
    if (!c.ssl) {
      *err = "SSL_new failed";
      return false;
    }
    SSL_set_fd(c.ssl, c.fd);
    const bool ip = is_ip_literal(host);
    if (!ip) SSL_set_tlsext_host_name(c.ssl, host.c_str());
    if (!opt.insecure_skip_verify) {
      // the chain must be valid AND issued for this server: its DNS name
      // (SAN / CN) or, for an IP master, its IP SAN
      X509_VERIFY_PARAM* vp = SSL_get0_param(c.ssl);
      X509_VERIFY_PARAM_set_hostflags(vp, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS);
      const int set = ip ? X509_VERIFY_PARAM_set1_ip_asc(vp, host.c_str()) : SSL_set1_host(c.ssl, host.c_str());
      if (set != 1) {
        *err = "cannot set the expected TLS peer name " + host;
        return false;
      }
    }
    if (SSL_connect(c.ssl) != 1) {
      const long vr = SSL_get_verify_result(c.ssl);
      *err = "TLS handshake with " + host + " failed" +
             (vr != X509_V_OK ? std::string(": ") + X509_verify_cert_error_string(vr) : std::string());
      ERR_clear_error();
      return false;
    }
#else
    *err = "https requested but pdo was built without OpenSSL";
    return false;
#endif
  }
  return true;
}

struct Head {
  int status = 0;
  std::map<std::string, std::string> headers;
};

void parse_head(const std::string& text, Head* h) {
  std::istringstream hs(text);
  std::string line;
  std::getline(hs, line);
  std::istringstream sl(line);
  std::string ver;
  sl >> ver >> h->status;
  while (std::getline(hs, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string v = line.substr(colon + 1);
    v.erase(0, v.find_first_not_of(' '));
    h->headers[lower(line.substr(0, colon))] = v;
  }
}

// one attempt on connection `c`.  *unsent = the request could not be written
// (never reached the server: always safe to send again); *no_answer = it was
// written but the server answered nothing at all (a stale keep-alive connection
// — or a server that applied it and then dropped the connection)
ClientResponse exchange(Conn& c, const std::string& req, const std::function<bool(const std::string&)>* on_line,
                        bool* unsent, bool* no_answer, bool* reusable) {
  ClientResponse out;
  *unsent = false;
  *no_answer = false;
  *reusable = false;
  if (!c.wr(req)) {
    *unsent = true;
    out.error = "send failed";
    return out;
  }
  std::string buf;
  char tmp[16384];
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t r = c.rd(tmp, sizeof tmp);
    if (r <= 0) {
      *no_answer = buf.empty();
      out.error = "no response";
      return out;
    }
    buf.append(tmp, (size_t)r);
  }
  Head h;
  parse_head(buf.substr(0, hdr_end), &h);
  out.status = h.status;
  out.headers = std::move(h.headers);
  buf.erase(0, hdr_end + 4);
  const bool chunked = lower(out.headers["transfer-encoding"]).find("chunked") != std::string::npos;
  const bool has_len = out.headers.count("content-length") > 0;
  const size_t clen = has_len ? (size_t)atol(out.headers["content-length"].c_str()) : 0;
  std::string linebuf;
  bool stop = false, complete = false;
  auto deliver = [&](const std::string& data) {
    if (!on_line) {
      out.body += data;
      return;
    }
    linebuf += data;
    size_t nl;
    while (!stop && (nl = linebuf.find('\n')) != std::string::npos) {
      std::string l = linebuf.substr(0, nl);
      linebuf.erase(0, nl + 1);
      if (!l.empty() && l.back() == '\r') l.pop_back();
      if (!l.empty() && !(*on_line)(l)) stop = true;
    }
  };
  auto fill = [&]() -> bool {
    ssize_t r = c.rd(tmp, sizeof tmp);
    if (r <= 0) return false;
    buf.append(tmp, (size_t)r);
    return true;
  };
  if (chunked) {
    while (!stop) {
      size_t crlf;
      while ((crlf = buf.find("\r\n")) == std::string::npos)
        if (!fill()) goto end;
      size_t n = strtoul(buf.substr(0, crlf).c_str(), nullptr, 16);
      buf.erase(0, crlf + 2);
      if (n == 0) {
        // trailer section ends with an empty line
        while (buf.find("\r\n") == std::string::npos)
          if (!fill()) goto end;
        complete = buf.compare(0, 2, "\r\n") == 0;
        break;
      }
      while (buf.size() < n + 2)
        if (!fill()) goto end;
      deliver(buf.substr(0, n));
      buf.erase(0, n + 2);
    }
  } else if (has_len) {
    while (buf.size() < clen)
      if (!fill()) break;
    deliver(buf.substr(0, std::min(clen, buf.size())));
    complete = buf.size() == clen;
  } else if (out.status == 204 || out.status == 304) {
    complete = buf.empty();
  } else {
    deliver(buf);
    buf.clear();
    while (!stop && fill()) {
      deliver(buf);
      buf.clear();
    }
  }
end:
  if (on_line && !linebuf.empty() && !stop) (*on_line)(linebuf);
  *reusable = complete && lower(out.headers["connection"]) != "close";
  return out;
}

ClientResponse do_request(const std::string& method, const std::string& url, const std::string& body,
                          const ClientOptions& opt, const std::function<bool(const std::string&)>* on_line) {
  ClientResponse out;
  std::string scheme, host, path;
  int port;
  if (!parse_url(url, &scheme, &host, &port, &path)) {
    out.error = "bad url " + url;
    return out;
  }
  const bool pooled = opt.keep_alive && !on_line;
  std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + host + ":" + std::to_string(port) + "\r\n";
  bool has_ct = false;
  for (auto& kv : opt.headers) {
    req += kv.first + ": " + kv.second + "\r\n";
    if (lower(kv.first) == "content-type") has_ct = true;
  }
  if (!has_ct && !body.empty()) req += "Content-Type: application/json\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  req += pooled ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
  req += body;
  const std::string key = scheme + "://" + host + ":" + std::to_string(port) + "#" +
                          std::to_string(std::hash<std::string>{}(tls_identity(opt)));
  for (int attempt = 0; attempt < 2; ++attempt) {
    std::unique_ptr<Conn> c = pooled ? pool_take(key) : nullptr;
    const bool reused = c != nullptr;
    if (!c) {
      c.reset(new Conn);
      if (!dial(*c, scheme, host, port, opt, &out.error)) return out;
      c->pool_key = key;
    } else {
      c->set_timeout(opt.timeout_s);
    }
    bool unsent = false, no_answer = false, reusable = false;
    out = exchange(*c, req, on_line, &unsent, &no_answer, &reusable);
    // a reused connection the server had already dropped: resend on a fresh one
    // only when the request never left, or repeating it is harmless
    const bool idem = opt.idempotent || method == "GET" || method == "HEAD" || method == "OPTIONS";
    if (out.status == 0 && reused && (unsent || (no_answer && idem))) continue;
    if (pooled && reusable) pool_put(std::move(c));
    return out;
  }
  return out;
}

// ------------------------------------------------------------------ SHA-1 (RFC 3174; WebSocket handshake only)
std::string sha1(const std::string& msg) {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  std::string m = msg;
  const uint64_t bits = (uint64_t)msg.size() * 8;
  m.push_back((char)0x80);
  while (m.size() % 64 != 56) m.push_back(0);
  for (int i = 7; i >= 0; --i) m.push_back((char)(bits >> (8 * i)));
  auto rol = [](uint32_t x, int n) { return (x << n) | (x >> (32 - n)); };
  for (size_t off = 0; off < m.size(); off += 64) {
    uint32_t w[80];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)(uint8_t)m[off + 4 * i] << 24 | (uint32_t)(uint8_t)m[off + 4 * i + 1] << 16 |
             (uint32_t)(uint8_t)m[off + 4 * i + 2] << 8 | (uint32_t)(uint8_t)m[off + 4 * i + 3];
    for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; ++i) {
      uint32_t f, k;
      if (i < 20) f = (b & c) | (~b & d), k = 0x5A827999u;
      else if (i < 40) f = b ^ c ^ d, k = 0x6ED9EBA1u;
      else if (i < 60) f = (b & c) | (b & d) | (c & d), k = 0x8F1BBCDCu;
      else f = b ^ c ^ d, k = 0xCA62C1D6u;
      const uint32_t t = rol(a, 5) + f + e + k + w[i];
      e = d, d = c, c = rol(b, 30), b = a, a = t;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e;
  }
  std::string out;
  for (uint32_t x : h)
    for (int i = 3; i >= 0; --i) out.push_back((char)(x >> (8 * i)));
  return out;
}

// ------------------------------------------------------------------ WebSocket framing (RFC 6455 §5)
std::string make_frame(int opcode, const std::string& pl, bool mask) {
  std::string f;
  f.push_back((char)(0x80 | (opcode & 0x0f)));
  const unsigned char mbit = mask ? 0x80 : 0;
  const uint64_t n = pl.size();
  if (n < 126) {
    f.push_back((char)(mbit | n));
  } else if (n < 65536) {
    f.push_back((char)(mbit | 126));
    f.push_back((char)(n >> 8));
    f.push_back((char)(n & 0xff));
  } else {
    f.push_back((char)(mbit | 127));
    for (int i = 7; i >= 0; --i) f.push_back((char)(n >> (8 * i)));
  }
  if (!mask) return f + pl;
  static thread_local std::mt19937 rng{std::random_device{}()};
  const uint32_t k = rng();
  const char key[4] = {(char)(k >> 24), (char)(k >> 16), (char)(k >> 8), (char)k};
  f.append(key, 4);
  for (size_t i = 0; i < pl.size(); ++i) f.push_back((char)(pl[i] ^ key[i & 3]));
  return f;
}

// one frame out of `buf`, refilled by fill(); payload unmasked
bool parse_frame(std::string& buf, const std::function<bool()>& fill, bool* fin, int* opcode, std::string* pl) {
  auto need = [&](size_t n) {
    while (buf.size() < n)
      if (!fill()) return false;
    return true;
  };
  if (!need(2)) return false;
  const unsigned char b0 = (unsigned char)buf[0], b1 = (unsigned char)buf[1];
  *fin = (b0 & 0x80) != 0;
  *opcode = b0 & 0x0f;
  const bool masked = (b1 & 0x80) != 0;
  uint64_t len = b1 & 0x7f;
  size_t hdr = 2;
  if (len == 126) {
    if (!need(4)) return false;
    len = (uint64_t)(unsigned char)buf[2] << 8 | (unsigned char)buf[3];
    hdr = 4;
  } else if (len == 127) {
    if (!need(10)) return false;
    len = 0;
    for (int i = 0; i < 8; ++i) len = len << 8 | (unsigned char)buf[2 + i];
    hdr = 10;
  }
  if (len > (64ull << 20)) return false;  // 64 MiB per frame is far beyond any exec stream chunk
  const size_t mk = hdr;
  if (masked) hdr += 4;
  if (!need(hdr + (size_t)len)) return false;
  pl->assign(buf, hdr, (size_t)len);
  if (masked)
    for (size_t i = 0; i < pl->size(); ++i) (*pl)[i] = (char)((*pl)[i] ^ buf[mk + (i & 3)]);
  buf.erase(0, hdr + (size_t)len);
  return true;
}

// one message: continuation frames reassembled, pings answered through pong()
bool read_message(std::string& buf, const std::function<bool()>& fill, const std::function<bool(const std::string&)>& pong,
                  int* opcode, std::string* msg) {
  msg->clear();
  int first = -1;
  while (true) {
    bool fin;
    int op;
    std::string pl;
    if (!parse_frame(buf, fill, &fin, &op, &pl)) return false;
    if (op == kWsPing) {
      if (!pong(pl)) return false;
      continue;
    }
    if (op == kWsPong) continue;
    if (op == kWsClose) {
      *opcode = kWsClose;
      *msg = pl;
      return true;
    }
    if (first < 0) first = op;
    *msg += pl;
    if (fin) {
      *opcode = first;
      return true;
    }
  }
}

}  // namespace

ClientResponse request(const std::string& method, const std::string& url, const std::string& body,
                       const ClientOptions& opt) {
  return do_request(method, url, body, opt, nullptr);
}

ClientResponse stream_lines(const std::string& method, const std::string& url, const std::string& body,
                            const std::function<bool(const std::string&)>& on_line, const ClientOptions& opt) {
  return do_request(method, url, body, opt, &on_line);
}

std::string ws_accept_key(const std::string& client_key) {
  return b64encode(sha1(client_key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"));
}

bool WsConn::send(int opcode, const std::string& payload) {
  const std::string f = make_frame(opcode, payload, false);
  return send_all(fd_, f.data(), f.size());
}

bool WsConn::recv(int* opcode, std::string* payload, double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  auto fill = [&]() -> bool {
    const double left =
        std::chrono::duration<double>(deadline - std::chrono::steady_clock::now()).count();
    if (left <= 0) return false;
    pollfd p{fd_, POLLIN, 0};
    if (::poll(&p, 1, (int)(left * 1000) + 1) != 1) return false;
    char tmp[16384];
    ssize_t r = ::recv(fd_, tmp, sizeof tmp, 0);
    if (r <= 0) return false;
    buf_.append(tmp, (size_t)r);
    return true;
  };
  auto pong = [&](const std::string& pl) { return send(kWsPong, pl); };
  return read_message(buf_, fill, pong, opcode, payload);
}

ExecResult ws_exec(const std::string& url, const ClientOptions& opt) {
  ExecResult r;
  std::string scheme, host, path;
  int port;
  if (!parse_url(url, &scheme, &host, &port, &path)) {
    r.error = "bad url " + url;
    return r;
  }
  if (scheme == "ws") scheme = "http";
  if (scheme == "wss") scheme = "https";
  Conn c;
  if (!dial(c, scheme, host, port, opt, &r.error)) return r;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(opt.timeout_s);
  std::string nonce(16, '\0');
  {
    static thread_local std::mt19937 rng{std::random_device{}()};
    for (auto& ch : nonce) ch = (char)(rng() & 0xff);
  }
  const std::string key = b64encode(nonce);
  std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host + ":" + std::to_string(port) + "\r\n";
  for (auto& kv : opt.headers) req += kv.first + ": " + kv.second + "\r\n";
  req += "Connection: Upgrade\r\nUpgrade: websocket\r\nSec-WebSocket-Version: 13\r\nSec-WebSocket-Key: " + key +
         "\r\nSec-WebSocket-Protocol: v5.channel.k8s.io, v4.channel.k8s.io\r\n\r\n";
  if (!c.wr(req)) {
    r.error = "send failed";
    return r;
  }
  std::string buf;
  char tmp[16384];
  auto fill = [&]() -> bool {
    if (std::chrono::steady_clock::now() > deadline) return false;
    ssize_t n = c.rd(tmp, sizeof tmp);
    if (n <= 0) return false;
    buf.append(tmp, (size_t)n);
    return true;
  };
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos)
    if (!fill()) {
      r.error = "no upgrade response";
      return r;
    }
  Head h;
  parse_head(buf.substr(0, hdr_end), &h);
  buf.erase(0, hdr_end + 4);
  if (h.status != 101) {
    r.error = "exec upgrade refused: HTTP " + std::to_string(h.status) + " " + buf.substr(0, 300);
    return r;
  }
  if (lower(h.headers["upgrade"]) != "websocket" || h.headers["sec-websocket-accept"] != ws_accept_key(key)) {
    r.error = "bad WebSocket handshake (Upgrade / Sec-WebSocket-Accept)";
    return r;
  }
  r.protocol = h.headers["sec-websocket-protocol"];
  auto pong = [&](const std::string& pl) { return c.wr(make_frame(kWsPong, pl, true)); };
  while (true) {
    int op;
    std::string msg;
    if (!read_message(buf, fill, pong, &op, &msg)) break;  // EOF / timeout
    if (op == kWsClose) break;
    if (msg.empty()) continue;
    const unsigned char ch = (unsigned char)msg[0];
    if (ch == 1) r.out.append(msg, 1, std::string::npos);
    else if (ch == 2) r.err.append(msg, 1, std::string::npos);
    else if (ch == 3) r.status.append(msg, 1, std::string::npos);
  }
  std::string code = "\x03\xe8";  // 1000 normal closure
  c.wr(make_frame(kWsClose, code, true));
  if (r.status.empty()) {
    r.error = std::chrono::steady_clock::now() > deadline ? "exec timed out" : "exec stream ended without a Status";
    return r;
  }
  // metav1.Status on the error channel: Success, or Failure with an ExitCode cause
  json::Value st;
  try {
    st = json::Value::parse(r.status);
  } catch (const std::exception& e) {
    r.error = std::string("bad exec Status: ") + e.what();
    return r;
  }
  if (st.get("status").str() == "Success") {
    r.ok = true;
    r.exit_code = 0;
    return r;
  }
  for (auto& cause : st.at_path("details.causes").arr())
    if (cause.get("reason").str() == "ExitCode") r.exit_code = atoi(cause.get("message").str().c_str());
  r.error = st.get("message").str("exec failed");
  return r;
}

}  // namespace http
}  // namespace pdo
