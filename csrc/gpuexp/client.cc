#include "gpuexp/client.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <strings.h>

#include <algorithm>
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

// Case-insensitive search for a header name inside [p, end); returns its value start.
const char* find_header(const char* p, const char* end, const char* name) {
  const size_t nl = std::strlen(name);
  for (; p + nl <= end; ++p) {
    if (p[0] != '\n') continue;
    const char* h = p + 1;
    if (size_t(end - h) < nl) break;
    if (::strncasecmp(h, name, nl) == 0) return h + nl;
  }
  return nullptr;
}

// Reads one HTTP response into `rb`, straight from the socket: one copy kernel -> user,
// no staging buffer, so the measured latency is the exporter's plus loopback TCP, not
// the harness's memcpys (a multi-GPU exposition is ~100-200 KB).  Returns the status
// code or -1; the body is [*body_off, *body_off + *body_len) of rb.data.
int read_response(int fd, RecvBuf* rb, size_t* body_off, size_t* body_len, bool* server_close) {
  auto fill = [&]() -> ssize_t {
    if (rb->data.size() - rb->end < 16384) rb->data.resize(std::max<size_t>(rb->data.size() * 2, 1 << 16));
    ssize_t n = ::recv(fd, rb->data.data() + rb->end, rb->data.size() - rb->end, 0);
    if (n > 0) rb->end += size_t(n);
    return n;
  };
  const char* hdr_end_p = nullptr;
  for (size_t scanned = rb->start;;) {
    const char* base = rb->data.data();
    if (rb->end >= rb->start + 4) {
      const char* from = base + std::max(rb->start, scanned >= 3 ? scanned - 3 : 0);
      const char* hit = static_cast<const char*>(::memmem(from, size_t(base + rb->end - from), "\r\n\r\n", 4));
      if (hit) {
        hdr_end_p = hit;
        break;
      }
      scanned = rb->end;
    }
    if (fill() <= 0) return -1;
  }
  const char* base = rb->data.data();
  const size_t hdr_end = size_t(hdr_end_p - base);
  const char* hs = base + rb->start;
  int code = hdr_end - rb->start > 12 ? std::atoi(hs + 9) : -1;
  const bool http10 = ::strncasecmp(hs, "HTTP/1.0", 8) == 0;
  const char* conn = find_header(hs, hdr_end_p, "connection:");
  *server_close = http10 || (conn && ::strncasecmp(conn + std::strspn(conn, " "), "close", 5) == 0);
  const char* cl = find_header(hs, hdr_end_p, "content-length:");
  if (!cl) {
    // No length: the body runs to EOF (HTTP/1.0 servers such as prometheus_client's).
    for (;;) {
      ssize_t n = fill();
      if (n < 0) return -1;
      if (n == 0) break;
    }
    *body_off = hdr_end + 4;
    *body_len = rb->end - *body_off;
    rb->start = rb->end;
    *server_close = true;
    return code;
  }
  uint64_t clen = 0;
  const char* eol = static_cast<const char*>(std::memchr(cl, '\r', size_t(hdr_end_p + 2 - cl)));
  parse_u64(cl, size_t((eol ? eol : hdr_end_p) - cl), &clen);
  const size_t need = hdr_end + 4 + size_t(clen);
  if (rb->data.size() < need) rb->data.resize(need + (1 << 16));
  while (rb->end < need)
    if (fill() <= 0) return -1;
  *body_off = hdr_end + 4;
  *body_len = size_t(clen);
  rb->start = need;
  return code;
}

}  // namespace

ScrapeClient::ScrapeClient(std::string host, int port, std::string path, bool gzip, int timeout_ms,
                           const std::string& accept, bool timing)
    : host_(std::move(host)), path_(std::move(path)), port_(port), timeout_ms_(timeout_ms) {
  req_ = "GET " + path_ + " HTTP/1.1\r\nHost: " + host_ + "\r\nUser-Agent: gpuexp-bench\r\n";
  if (gzip) req_ += "Accept-Encoding: gzip\r\n";
  if (timing) req_ += "X-Gpuexp-Timing: 1\r\n";
  if (!accept.empty()) req_ += "Accept: " + accept + "\r\n";
  req_ += "\r\n";
}

ScrapeClient::~ScrapeClient() {
  if (fd_ >= 0) ::close(fd_);
}

double ScrapeClient::scrape() {
  if (fd_ < 0) {
    fd_ = connect_to(host_, port_, timeout_ms_);
    rb_.start = rb_.end = 0;
    if (fd_ < 0) {
      ++errors_;
      return -1;
    }
  }
  rb_.compact();
  uint64_t t0 = mono_ns();
  bool ok = ::send(fd_, req_.data(), req_.size(), MSG_NOSIGNAL) == ssize_t(req_.size());
  bool server_close = false;
  int code = ok ? read_response(fd_, &rb_, &body_off_, &body_len_, &server_close) : -1;
  uint64_t t1 = mono_ns();
  if (code < 0) {
    ++errors_;
    ::close(fd_);
    fd_ = -1;
    return -1;
  }
  status_ = code;
  bytes_ = body_len_;
  t_send_ = t0;
  t_done_ = t1;
  t_srv_parse_ = t_srv_write_ = 0;
  srv_prewoken_ = -1;
  t_srv_rx_ = 0;
  {
    // the response's header block ends 4 bytes before the body
    static const char kName[] = "\r\nX-Gpuexp-Timing: ";
    const char* hb = rb_.data.data();
    const char* he = hb + body_off_;
    const char* p = std::search(hb, he, kName, kName + sizeof(kName) - 1);
    if (p != he) {
      p += sizeof(kName) - 1;
      char* q = nullptr;
      t_srv_parse_ = std::strtoull(p, &q, 10);
      char* r = nullptr;
      t_srv_write_ = q ? std::strtoull(q, &r, 10) : 0;
      char* s2 = nullptr;
      srv_prewoken_ = r && *r == ' ' ? int(std::strtol(r, &s2, 10)) : -1;
      t_srv_rx_ = s2 && *s2 == ' ' ? std::strtoull(s2, nullptr, 10) : 0;
    }
  }
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
  RecvBuf rb;
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
      rb.start = rb.end = 0;
      if (fd < 0) {
        r.errors++;
        continue;
      }
    }
    rb.compact();
    size_t boff = 0, blen = 0;
    uint64_t t0 = mono_ns();
    bool ok = ::send(fd, req.data(), req.size(), MSG_NOSIGNAL) == ssize_t(req.size());
    bool server_close = false;
    int code = ok ? read_response(fd, &rb, &boff, &blen, &server_close) : -1;
    uint64_t t1 = mono_ns();
    if (code < 0) {
      r.errors++;
      ::close(fd);
      fd = -1;
      continue;
    }
    if (code != 200) r.non200++;
    r.latency_ns.push_back(double(t1 - t0));
    r.bytes += blen;
    if (keep_last_body) r.last_body.assign(rb.data.data() + boff, blen);
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
