// Small helpers shared by the engine's translation units (engine*.cc).  Internal header.
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <string>
#include <vector>

namespace gpuexp {
namespace engine_util {

inline std::string lower(std::string s) {
  std::transform(s.begin(), s.end(), s.begin(), ::tolower);
  return s;
}

// Delta of a monotonically increasing hardware accumulator.  Unsigned wrap is accepted
// when the wrapped delta is plausible; a large backwards jump is a reset (returns false).
inline bool acc_delta(uint64_t cur, uint64_t prev, double* d) {
  const uint64_t diff = cur - prev;  // modular
  if (cur >= prev || diff < (1ull << 62)) {
    *d = double(diff);
    return true;
  }
  return false;
}

// "0".."63" without a std::to_string per series per tick (label values of links / XCDs)
inline const char* idx_str(int i) {
  static const char* k[64] = {"0",  "1",  "2",  "3",  "4",  "5",  "6",  "7",  "8",  "9",  "10", "11", "12",
                              "13", "14", "15", "16", "17", "18", "19", "20", "21", "22", "23", "24", "25",
                              "26", "27", "28", "29", "30", "31", "32", "33", "34", "35", "36", "37", "38",
                              "39", "40", "41", "42", "43", "44", "45", "46", "47", "48", "49", "50", "51",
                              "52", "53", "54", "55", "56", "57", "58", "59", "60", "61", "62", "63"};
  return i >= 0 && i < 64 ? k[i] : "?";
}

}  // namespace engine_util
}  // namespace gpuexp
