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

#include <algorithm>
#include <cctype>
#include <cstring>
#include <sstream>

#ifdef PDO_WITH_TLS
#include <openssl/err.h>
#include <openssl/ssl.h>
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

static const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
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
  fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
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
  ::shutdown(fd_, SHUT_RDWR);
  ::close(fd_);
  fd_ = -1;
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int cfd : conn_fds_) ::shutdown(cfd, SHUT_RDWR);
  }
  // connection threads are detached; wait (bounded) for them to leave
  for (int i = 0; i < 500 && active_.load() > 0; ++i) usleep(2000);
}

void Server::accept_loop() {
  while (running_) {
    sockaddr_in sa{};
    socklen_t len = sizeof sa;
    int cfd = ::accept(fd_, (sockaddr*)&sa, &len);
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
struct Conn {
  int fd = -1;
#ifdef PDO_WITH_TLS
  SSL_CTX* ctx = nullptr;
  SSL* ssl = nullptr;
#endif
  ~Conn() {
#ifdef PDO_WITH_TLS
    if (ssl) {
      SSL_shutdown(ssl);
      SSL_free(ssl);
    }
    if (ctx) SSL_CTX_free(ctx);
#endif
    if (fd >= 0) ::close(fd);
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
};

bool dial(Conn& c, const std::string& scheme, const std::string& host, int port, const ClientOptions& opt,
          std::string* err) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
    *err = "resolve " + host + " failed";
    return false;
  }
  for (addrinfo* a = res; a; a = a->ai_next) {
    c.fd = ::socket(a->ai_family, a->ai_socktype, a->ai_protocol);
    if (c.fd < 0) continue;
    timeval tv;
    tv.tv_sec = (long)opt.timeout_s;
    tv.tv_usec = (long)((opt.timeout_s - (long)opt.timeout_s) * 1e6);
    setsockopt(c.fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(c.fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (::connect(c.fd, a->ai_addr, a->ai_addrlen) == 0) break;
    ::close(c.fd);
    c.fd = -1;
  }
  freeaddrinfo(res);
  if (c.fd < 0) {
    *err = "connect " + host + ":" + std::to_string(port) + " failed";
    return false;
  }
  int one = 1;
  setsockopt(c.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  if (scheme == "https") {
#ifdef PDO_WITH_TLS
    c.ctx = SSL_CTX_new(TLS_client_method());
    if (!opt.ca_file.empty()) SSL_CTX_load_verify_locations(c.ctx, opt.ca_file.c_str(), nullptr);
    else SSL_CTX_set_default_verify_paths(c.ctx);
    SSL_CTX_set_verify(c.ctx, opt.insecure_skip_verify ? SSL_VERIFY_NONE : SSL_VERIFY_PEER, nullptr);
    if (!opt.cert_file.empty()) SSL_CTX_use_certificate_file(c.ctx, opt.cert_file.c_str(), SSL_FILETYPE_PEM);
    if (!opt.key_file.empty()) SSL_CTX_use_PrivateKey_file(c.ctx, opt.key_file.c_str(), SSL_FILETYPE_PEM);
    c.ssl = SSL_new(c.ctx);
    SSL_set_fd(c.ssl, c.fd);
    SSL_set_tlsext_host_name(c.ssl, host.c_str());
    if (SSL_connect(c.ssl) != 1) {
      *err = "TLS handshake with " + host + " failed";
      return false;
    }
#else
    *err = "https requested but pdo was built without OpenSSL";
    return false;
#endif
  }
  return true;
}

// reads a full response; if on_line is set, streams the body line by line
ClientResponse do_request(const std::string& method, const std::string& url, const std::string& body,
                          const ClientOptions& opt, const std::function<bool(const std::string&)>* on_line) {
  ClientResponse out;
  std::string scheme, host, path;
  int port;
  if (!parse_url(url, &scheme, &host, &port, &path)) {
    out.error = "bad url " + url;
    return out;
  }
  Conn c;
  if (!dial(c, scheme, host, port, opt, &out.error)) return out;
  std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + host + ":" + std::to_string(port) + "\r\n";
  bool has_ct = false;
  for (auto& kv : opt.headers) {
    req += kv.first + ": " + kv.second + "\r\n";
    if (lower(kv.first) == "content-type") has_ct = true;
  }
  if (!has_ct && !body.empty()) req += "Content-Type: application/json\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
  if (!c.wr(req)) {
    out.error = "send failed";
    return out;
  }
  std::string buf;
  char tmp[16384];
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t r = c.rd(tmp, sizeof tmp);
    if (r <= 0) {
      out.error = "no response";
      return out;
    }
    buf.append(tmp, (size_t)r);
  }
  {
    std::istringstream hs(buf.substr(0, hdr_end));
    std::string line;
    std::getline(hs, line);
    std::istringstream sl(line);
    std::string ver;
    sl >> ver >> out.status;
    while (std::getline(hs, line)) {
      if (!line.empty() && line.back() == '\r') line.pop_back();
      size_t colon = line.find(':');
      if (colon == std::string::npos) continue;
      std::string v = line.substr(colon + 1);
      v.erase(0, v.find_first_not_of(' '));
      out.headers[lower(line.substr(0, colon))] = v;
    }
  }
  buf.erase(0, hdr_end + 4);
  const bool chunked = lower(out.headers["transfer-encoding"]).find("chunked") != std::string::npos;
  const bool has_len = out.headers.count("content-length") > 0;
  const size_t clen = has_len ? (size_t)atol(out.headers["content-length"].c_str()) : 0;
  std::string linebuf;
  bool stop = false;
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
      if (n == 0) break;
      while (buf.size() < n + 2)
        if (!fill()) goto end;
      deliver(buf.substr(0, n));
      buf.erase(0, n + 2);
    }
  } else if (has_len) {
    while (buf.size() < clen)
      if (!fill()) break;
    deliver(buf.substr(0, std::min(clen, buf.size())));
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
  return out;
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

}  // namespace http
}  // namespace pdo
