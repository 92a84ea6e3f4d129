// Keep-alive HTTP scrape client used by the benchmark harness: paced at a fixed rate
// (absolute-deadline clock_nanosleep), timing each GET from just before send() to the
// last body byte, so the measured latency excludes Python interpreter overhead.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace gpuexp {

struct ScrapeResult {
  std::vector<double> latency_ns;
  uint64_t bytes = 0;
  uint64_t errors = 0;
  uint64_t non200 = 0;
  std::string last_body;
  double wall_s = 0;
};

// Receive buffer reused across responses: [start, end) holds unread bytes.
struct RecvBuf {
  std::vector<char> data = std::vector<char>(size_t(1) << 18);
  size_t start = 0, end = 0;
  // Moves unread bytes (a pipelined response, normally none) to the front.
  void compact() {
    if (start == 0) return;
    std::copy(data.begin() + long(start), data.begin() + long(end), data.begin());
    end -= start;
    start = 0;
  }
};

// One persistent keep-alive connection; scrape() returns the latency in ns (-1 on error).
class ScrapeClient {
 public:
  // accept: optional Accept header value (e.g. the protobuf exposition's media type).
  // timing: ask the server to echo its timestamps (X-Gpuexp-Timing) for a latency split.
  ScrapeClient(std::string host, int port, std::string path, bool gzip, int timeout_ms,
               const std::string& accept = "", bool timing = false);
  ~ScrapeClient();
  double scrape();
  int last_status() const { return status_; }
  uint64_t last_bytes() const { return bytes_; }
  // Body of the last response (valid until the next scrape).
  std::string last_body() const { return std::string(rb_.data.data() + body_off_, body_len_); }
  uint64_t errors() const { return errors_; }
  // Last scrape, CLOCK_MONOTONIC ns: {client send, server parsed, server writing, client done};
  // the server fields are 0 unless timing was requested and echoed.
  std::vector<uint64_t> last_timing() const { return {t_send_, t_srv_parse_, t_srv_write_, t_done_}; }
  // 1 if the server's worker was pre-woken for the last request, 0 if not, -1 unknown.
  int last_prewoken() const { return srv_prewoken_; }
  // CLOCK_MONOTONIC ns at which the server's kernel queued the request (0 = not known).
  uint64_t last_server_rx() const { return t_srv_rx_; }

 private:
  uint64_t t_send_ = 0, t_srv_parse_ = 0, t_srv_write_ = 0, t_done_ = 0;
  int srv_prewoken_ = -1;
  uint64_t t_srv_rx_ = 0;
  std::string host_, path_, req_;
  int port_, timeout_ms_, fd_ = -1, status_ = 0;
  uint64_t bytes_ = 0, errors_ = 0;
  RecvBuf rb_;
  size_t body_off_ = 0, body_len_ = 0;
};

ScrapeResult scrape_loop(const std::string& host, int port, const std::string& path, double hz, int count,
                         bool gzip, bool keepalive, int timeout_ms, bool keep_last_body);

}  // namespace gpuexp
