// Immutable exposition snapshots, published by the sampler and pinned by scrapers.
//
// The reference rendered inside the scrape (promhttp Gather, main.go:68-70) with the
// two GaugeVecs updated concurrently by the collection loop (main.go:147-150), so a
// scrape could see a new bytes value next to an old percent value.
// Here one tick renders ALL families into one body; publication is a single
// seq_cst store of the slot index, and readers pin a slot with a refcount, so a scrape
// never blocks the sampler and always sees one consistent tick.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace gpuexp {

struct Snapshot {
  std::string body;     // text 0.0.4
  std::string gz;       // gzip(body), empty when not produced for this tick
  std::string pb;       // delimited MetricFamily protobuf, only while scrapers negotiate it
  std::string pb_gz;    // gzip(pb), only while protobuf + gzip are both asked for
  uint64_t gen = 0;     // sampler generation that produced it
  uint64_t render_ns = 0;
  uint64_t series = 0;
  uint64_t published_mono_ns = 0;  // CLOCK_MONOTONIC at publication (staleness checks)
};

class SnapshotStore {
 public:
  static constexpr int kSlots = 8;

  class Pin {
   public:
    Pin() = default;
    Pin(SnapshotStore* st, int slot) : st_(st), slot_(slot) {}
    Pin(const Pin&) = delete;
    Pin& operator=(const Pin&) = delete;
    Pin(Pin&& o) noexcept : st_(o.st_), slot_(o.slot_) { o.st_ = nullptr; o.slot_ = -1; }
    Pin& operator=(Pin&& o) noexcept {
      release();
      st_ = o.st_;
      slot_ = o.slot_;
      o.st_ = nullptr;
      o.slot_ = -1;
      return *this;
    }
    ~Pin() { release(); }
    explicit operator bool() const { return slot_ >= 0; }
    const Snapshot* operator->() const { return &st_->slots_[slot_].snap; }
    const Snapshot& operator*() const { return st_->slots_[slot_].snap; }
    void release() {
      if (st_ && slot_ >= 0) st_->slots_[slot_].refs.fetch_sub(1, std::memory_order_seq_cst);
      st_ = nullptr;
      slot_ = -1;
    }

   private:
    SnapshotStore* st_ = nullptr;
    int slot_ = -1;
  };

  // Reader side: any thread.  Returns an empty pin before the first publish.
  Pin acquire() {
    for (;;) {
      int c = current_.load(std::memory_order_seq_cst);
      if (c < 0) return Pin();
      slots_[c].refs.fetch_add(1, std::memory_order_seq_cst);
      if (current_.load(std::memory_order_seq_cst) == c) return Pin(this, c);
      slots_[c].refs.fetch_sub(1, std::memory_order_seq_cst);
    }
  }

  // Writer side: single thread.  Returns a free slot (not current, not pinned) or -1
  // if every other slot is pinned by slow readers (the tick is then not published).
  // Prefers the slot published before the current one: slots ping-pong while scrapes are
  // quick, so the render writes into buffers touched one tick ago (still in cache) rather
  // than cycling through all kSlots cold ones.
  int begin_write() {
    int c = current_.load(std::memory_order_seq_cst);
    if (prev_ >= 0 && prev_ != c && slots_[prev_].refs.load(std::memory_order_seq_cst) == 0) return prev_;
    for (int k = 1; k <= kSlots; ++k) {
      int i = (c + k + kSlots) % kSlots;
      if (i == c) continue;
      if (slots_[i].refs.load(std::memory_order_seq_cst) == 0) return i;
    }
    return -1;
  }
  Snapshot* slot(int i) { return &slots_[i].snap; }
  void publish(int i) {
    prev_ = current_.load(std::memory_order_seq_cst);
    current_.store(i, std::memory_order_seq_cst);
  }
  bool ready() const { return current_.load(std::memory_order_acquire) >= 0; }

 private:
  struct alignas(64) Slot {
    std::atomic<int> refs{0};
    Snapshot snap;
  };
  Slot slots_[kSlots];
  std::atomic<int> current_{-1};
  int prev_ = -1;  // writer thread only
};

// gzip (RFC 1952) of `in` at compression `level` into `out`.  Returns false on error.
bool gzip_compress(const std::string& in, std::string* out, int level = 1);
// "libdeflate" (loaded at run time when present) or "zlib".
const char* gzip_impl();

}  // namespace gpuexp
