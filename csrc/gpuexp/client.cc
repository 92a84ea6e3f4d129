#include "gpuexp/client.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "gpuexp/common.h"

namespace gpuexp {

namespace {

int connect_to(const std::string& host, int port, int timeout_ms) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  if (::inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1 ||
      ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

// Reads one HTTP response; returns status code or -1.  `buf` may hold leftover bytes.
int read_response(int fd, std::string* buf, std::string* body, bool* server_close) {
  char tmp[65536];
  size_t hdr_end;
  while ((hdr_end = buf->find("\r\n\r\n")) == std::string::npos) {
    ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return -1;
    buf->append(tmp, size_t(n));
  }
  int code = -1;
  if (buf->size() > 12) code = std::atoi(buf->c_str() + 9);
  uint64_t clen = 0;
  std::string headers = buf->substr(0, hdr_end);
  for (auto& c : headers) c = char(::tolower(c));
  size_t p = headers.find("content-length:");
  bool http10 = headers.compare(0, 8, "http/1.0") == 0;
  *server_close = http10 || headers.find("connection: close") != std::string::npos;
  if (p == std::string::npos) {
    // No length: the body runs to EOF (HTTP/1.0 servers such as prometheus_client's).
    for (;;) {
      ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
      if (n < 0) return -1;
      if (n == 0) break;
      buf->append(tmp, size_t(n));
    }
    body->assign(*buf, hdr_end + 4, std::string::npos);
    buf->clear();
    *server_close = true;
    return code;
  }
  parse_u64(headers.c_str() + p + 15, headers.size() - p - 15, &clen);
  size_t need = hdr_end + 4 + size_t(clen);
  while (buf->size() < need) {
    ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return -1;
    buf->append(tmp, size_t(n));
  }
  body->assign(*buf, hdr_end + 4, size_t(clen));
  buf->erase(0, need);
  return code;
}

}  // namespace

ScrapeClient::ScrapeClient(std::string host, int port, std::string path, bool gzip, int timeout_ms,
                           const std::string& accept)
    : host_(std::move(host)), path_(std::move(path)), port_(port), timeout_ms_(timeout_ms) {
  req_ = "GET " + path_ + " HTTP/1.1\r\nHost: " + host_ + "\r\nUser-Agent: gpuexp-bench\r\n";
  if (gzip) req_ += "Accept-Encoding: gzip\r\n";
  if (!accept.empty()) req_ += "Accept: " + accept + "\r\n";
  req_ += "\r\n";
}

ScrapeClient::~ScrapeClient() {
  if (fd_ >= 0) ::close(fd_);
}

double ScrapeClient::scrape() {
  if (fd_ < 0) {
    fd_ = connect_to(host_, port_, timeout_ms_);
    buf_.clear();
    if (fd_ < 0) {
      ++errors_;
      return -1;
    }
  }
  uint64_t t0 = mono_ns();
  bool ok = ::send(fd_, req_.data(), req_.size(), MSG_NOSIGNAL) == ssize_t(req_.size());
  bool server_close = false;
  int code = ok ? read_response(fd_, &buf_, &body_, &server_close) : -1;
  uint64_t t1 = mono_ns();
  if (code < 0) {
    ++errors_;
    ::close(fd_);
    fd_ = -1;
    return -1;
  }
  status_ = code;
  bytes_ = body_.size();
  if (server_close) {
    ::close(fd_);
    fd_ = -1;
  }
  return double(t1 - t0);
}

ScrapeResult scrape_loop(const std::string& host, int port, const std::string& path, double hz, int count,
                         bool gzip, bool keepalive, int timeout_ms, bool keep_last_body) {
  ScrapeResult r;
  r.latency_ns.reserve(size_t(count > 0 ? count : 0));
  std::string req = "GET " + path + " HTTP/1.1\r\nHost: " + host + "\r\nUser-Agent: gpuexp-bench\r\n";
  if (gzip) req += "Accept-Encoding: gzip\r\n";
  req += keepalive ? "\r\n" : "Connection: close\r\n\r\n";
  int fd = -1;
  std::string buf, body;
  timespec next;
  clock_gettime(CLOCK_MONOTONIC, &next);
  uint64_t period_ns = hz > 0 ? uint64_t(1e9 / hz) : 0;
  uint64_t t_start = mono_ns();
  for (int i = 0; i < count; ++i) {
    if (period_ns) {
      clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &next, nullptr);
      uint64_t ns = uint64_t(next.tv_nsec) + period_ns;
      next.tv_sec += time_t(ns / 1000000000ull);
      next.tv_nsec = long(ns % 1000000000ull);
    }
    if (fd < 0) {
      fd = connect_to(host, port, timeout_ms);
      buf.clear();
      if (fd < 0) {
        r.errors++;
        continue;
      }
    }
    uint64_t t0 = mono_ns();
    bool ok = ::send(fd, req.data(), req.size(), MSG_NOSIGNAL) == ssize_t(req.size());
    bool server_close = false;
    int code = ok ? read_response(fd, &buf, &body, &server_close) : -1;
    uint64_t t1 = mono_ns();
    if (code < 0) {
      r.errors++;
      ::close(fd);
      fd = -1;
      continue;
    }
    if (code != 200) r.non200++;
    r.latency_ns.push_back(double(t1 - t0));
    r.bytes += body.size();
    if (keep_last_body) r.last_body = body;
    if (!keepalive || server_close) {
      ::close(fd);
      fd = -1;
    }
  }
  if (fd >= 0) ::close(fd);
  r.wall_s = double(mono_ns() - t_start) * 1e-9;
  return r;
}

}  // namespace gpuexp
