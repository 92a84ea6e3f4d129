// Prometheus text-format 0.0.4 series table + renderer.
//
// Reference: two client_golang GaugeVecs registered on a custom registry
// (/root/reference/main.go:21-36, :40-42) rendered by promhttp on every scrape
// (main.go:68-70).  Here every series owns a pre-rendered `name{labels} ` prefix that is
// built once when the label set is interned; a tick only formats numbers, and the
// result is published as an immutable snapshot that scrapes copy out with writev().
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "gpuexp/deflate_tmpl.h"

namespace gpuexp {

enum class MetricType : uint8_t { kGauge = 0, kCounter = 1, kHistogram = 2 };

struct FamilyDef {
  std::string name;
  std::string help;
  MetricType type = MetricType::kGauge;
  std::vector<std::string> label_names;
};

// Versioned handle: a slot freed by GC and reused for another label set bumps its
// version, so a stale cached handle is detected instead of writing a wrong series.
struct SeriesRef {
  uint32_t idx = UINT32_MAX;
  uint32_t ver = 0;
  bool valid() const { return idx != UINT32_MAX; }
};

// Appends `v` in the shortest round-trip form ("NaN", "+Inf", "-Inf" for specials;
// integers without exponent up to 2^53).
void append_value(std::string* out, double v);
// The same into buf (>= 40 bytes); returns the length.
size_t format_value(char* buf, double v);
void append_escaped_label_value(std::string* out, const std::string& v);
void append_escaped_help(std::string* out, const std::string& v);
bool valid_metric_name(const std::string& s);
bool valid_label_name(const std::string& s);

class SeriesTable {
 public:
  // Families render sorted by name (client_golang's Gather order).
  int add_family(const FamilyDef& def);
  int family_id(const std::string& name) const;
  const FamilyDef& family(int fid) const { return families_[size_t(fid)].def; }
  size_t num_families() const { return families_.size(); }

  // Interns (family, label values) and returns a handle.  Slow path (hashing); callers
  // cache handles for series that persist across ticks.
  SeriesRef upsert(int fid, const std::vector<std::string>& values);
  // Sets a gauge/counter value and marks the series live for generation `gen`.
  // Returns false if the handle went stale (caller must re-upsert).
  bool set(SeriesRef r, double v, uint64_t gen);
  // Histogram observation (cumulative; `bounds` fixed at first use).
  bool observe(SeriesRef r, double v, uint64_t gen, const std::vector<double>& bounds);
  // Marks a histogram series live without a new observation.
  bool touch(SeriesRef r, uint64_t gen);
  // Replaces a histogram's state wholesale (non-cumulative bucket counts; the last
  // entry of `counts` is the +Inf overflow and is implied by `count`).
  bool set_histogram(SeriesRef r, const std::vector<double>& bounds,
                     const std::vector<uint64_t>& counts, double sum, uint64_t count, uint64_t gen);

  // Convenience: upsert + set.
  void put(int fid, const std::vector<std::string>& values, double v, uint64_t gen) {
    set(upsert(fid, values), v, gen);
  }

  // Renders every series that is live at `gen`.  Series not live for more than
  // `gc_after` generations are freed (stale-series GC; the reference never Reset() its
  // vectors, main.go:147-150, so exited PIDs stayed forever).
  void render(std::string* out, uint64_t gen, uint64_t gc_after = 1);
  // The same live series as length-delimited io.prometheus.client.MetricFamily protobuf
  // messages (what client_golang's promhttp serves when a scraper negotiates
  // `application/vnd.google.protobuf; proto=io.prometheus.client.MetricFamily;
  // encoding=delimited`).  Call after render() of the same generation (GC + ordering).
  void render_proto(std::string* out, uint64_t gen) const;

  // Fixed-layout rendering: the samples render() gives, with every value right-aligned in a
  // blank-led field whose width only grows (per series), so the body keeps its layout from tick to tick.
  // Between layout changes (a series appears or goes, a value outgrows its field) a tick only
  // patches the fields whose values changed, and -- with `gz` -- emits the gzip member from the
  // pre-encoded static bits plus the field bytes (TemplateDeflate).  Do not mix with render()
  // on one table.
  // `out_gen`: the generation `out` holds a render_compiled body of (0 = none, e.g. a fresh
  // snapshot slot): if the layout has not changed since, only the fields changed after it are
  // copied into `out` instead of the whole body.
  void render_compiled(std::string* out, std::string* gz, uint64_t gen, uint64_t gc_after = 1,
                       uint64_t out_gen = 0);
  // Families laid out again by the last render_compiled (0 in steady state).
  size_t last_relayouts() const { return last_relayouts_; }
  size_t last_skipped() const { return last_skipped_; }
  size_t last_walked() const { return last_walked_; }
  // Segments encoded without matches while the layout settled (cumulative).
  uint64_t provisional_parses() const { return provisional_parses_; }
  // Bytes copied into `out` by the last render_compiled (the whole body, or the changed fields).
  size_t last_copied() const { return last_copied_; }
  uint64_t code_builds() const { return code_builds_; }
  const TemplateDeflate& deflater() const { return deflate_; }

  size_t live_series(uint64_t gen) const;
  // Families whose text was re-built by the last render (the rest were copied cached).
  size_t last_rebuilt_families() const { return last_rebuilt_; }
  size_t live_series_in_family(int fid, uint64_t gen) const;
  double value(SeriesRef r) const;

 private:
  // Per-series fields every tick touches, in their own dense array (hot_[idx]): setting
  // values, the GC/liveness scan and the render-cache check never walk the large Series
  // records, so a 10 Hz tick that starts with cold caches stays cheap.
  struct Hot {
    int fid = -1;
    uint32_t ver = 0;
    uint64_t gen = 0;       // last generation it was set
    double value = 0;
    bool in_cache = false;  // included in its family's cached text
    uint32_t stamp = 0;     // bumped on every value/histogram change (render_compiled)
    bool laid = false;      // a member of its family's compiled layout
  };
  // Per-family state every set() touches, dense by family id (a few KB: stays in cache through
  // the series stage), so render_compiled can pass over a family with no change without walking
  // its members.
  struct FamHot {
    uint64_t gen = 0;        // generation of the three counts below
    uint32_t live = 0;       // members set this generation
    uint32_t live_laid = 0;  // ... of which in the compiled layout
    uint32_t changed = 0;    // value / histogram changes this generation
    uint32_t nmembers = 0;
    uint32_t nlaid = 0;      // members in the compiled layout (laid_valid)
    bool laid_valid = false;
    bool dirty = true;       // render(): the cached text is stale
    bool dirty_order = false;
    uint64_t change_gen = 0;  // generation a field of the family was last written in (render_compiled)
  };
  struct Series {  // cold: strings and histogram state
    std::vector<std::string> labels;
    std::string prefix;       // `name{a="x",b="y"}` (no trailing space)
    std::string line;         // prefix + ' ' (what render copies before the value)
    std::string key;          // interning key
    // Formatted value cache: re-formatted only when the value's bits change (most device
    // series — identity, capacities, link state, error totals — change rarely).
    uint64_t vbits = 0;
    uint8_t vlen = 0;
    bool vvalid = false;
    char vtxt[32];
    // histogram state
    std::vector<double> bounds;
    std::vector<uint64_t> buckets;
    double hsum = 0;
    uint64_t hcount = 0;
    std::vector<std::string> hlines;  // `name_bucket{...,le="b"} ` per bound, +Inf, _sum, _count
    std::vector<uint8_t> widths;      // render_compiled field widths (value, or each histogram line)
  };
  struct Family {
    FamilyDef def;
    std::string header;              // "# HELP ...\n# TYPE ...\n"
    std::vector<uint32_t> members;   // sorted by label values (FamHot::dirty_order: not yet)
    // Rendered text of the family as of the last render.  Re-built only when a member's
    // value bits, membership or liveness changed (FamHot::dirty); otherwise render copies it.
    std::string cache;
  };
  // render_compiled state of one family: its live members as laid out, its segment of the
  // body, and per member the fields it owns and the stamp they were written with.
  struct LaidMember {
    uint32_t idx, ver;
    uint32_t stamp;        // the value stamp its fields were written with
    uint32_t first_field;  // fields of one member are contiguous
    uint64_t change_gen;   // generation its fields were last written in
  };
  struct Layout {
    bool valid = false;
    bool relayout = false;
    const char* why = "";  // why it is laid out again (GPUEXP_DEBUG_RELAYOUT logs it)
    std::vector<LaidMember> members;  // one array: the per-tick pass streams through it
    TmplSegment seg;
  };
  // Field texts of series `idx` (1 for a gauge/counter, bounds + 3 for a histogram) into
  // scratch_ / scratch_len_.
  void field_texts(uint32_t idx);
  void layout_family(int fid, uint64_t gen, std::string* body);
  void free_series(uint32_t idx);
  void sort_members(int fid);
  // bookkeeping of a set/observe/touch of series `h` at `gen` (changed: its value changed)
  void note_set(Hot& h, uint64_t gen, bool changed) {
    FamHot& f = fam_hot_[size_t(h.fid)];
    if (f.gen != gen) {
      f.gen = gen;
      f.live = f.live_laid = f.changed = 0;
    }
    if (h.gen != gen) {
      ++f.live;
      if (h.laid) ++f.live_laid;
      h.gen = gen;
    }
    if (changed) {
      ++f.changed;
      f.dirty = true;
      h.stamp += 1;
    }
  }
  void unlay(int fid);  // the family's compiled layout is gone: its members are no longer laid
  void render_histogram(std::string* out, uint32_t idx);
  void build_hlines(uint32_t idx);
  void format_cached(uint32_t idx);  // (re)fills the series' vtxt cache
  void append_cached_value(std::string* out, uint32_t idx);
  void mark_dirty(int fid) { fam_hot_[size_t(fid)].dirty = true; }

  std::vector<Family> families_;
  std::vector<FamHot> fam_hot_;  // by family id
  std::vector<int> render_order_;  // family ids sorted by name
  std::vector<Hot> hot_;
  std::vector<Series> series_;
  std::vector<uint32_t> free_;
  std::unordered_map<std::string, uint32_t> index_;
  std::string keybuf_;
  size_t last_rebuilt_ = 0;
  // render_compiled
  std::vector<Layout> layouts_;  // by family id
  std::string cbody_, cbody_next_;
  std::vector<TmplSegment*> csegs_;
  TemplateDeflate deflate_;
  size_t last_relayouts_ = 0;
  uint64_t compiled_gen_ = 0;  // generation of the last render_compiled
  bool parse_check_ = true;    // segments were laid out since their parses were last checked
  bool debug_relayout_ = false;  // GPUEXP_DEBUG_RELAYOUT: log every family laid out again (stderr)
  uint64_t rebuild_gen_ = 0;   // generation of the last layout change
  size_t last_copied_ = 0;
  uint64_t provisional_parses_ = 0;  // segments parsed on their own while their layout settled
  static constexpr uint64_t kStableRenders = 3;
  static constexpr size_t kLookback = 8192;  // how far a segment's matches may reach back
  size_t last_skipped_ = 0;    // families passed over unchanged by the last render_compiled
  size_t last_walked_ = 0;     // families whose members the last render_compiled walked
  uint64_t code_builds_ = 0;
  size_t relaid_bytes_ = 0;  // bytes (re-)parsed since the code was last built
  std::vector<char> scratch_;  // field_texts output, 32 bytes per field
  std::vector<uint8_t> scratch_len_;
};

}  // namespace gpuexp
