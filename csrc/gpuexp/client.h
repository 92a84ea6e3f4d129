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

ScrapeResult scrape_loop(const std::string& host, int port, const std::string& path, double hz, int count,
                         bool gzip, bool keepalive, int timeout_ms, bool keep_last_body);

}  // namespace gpuexp
