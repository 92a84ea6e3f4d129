#include "gpuexp/exposition.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <stdexcept>

namespace gpuexp {

size_t format_value(char* buf, double v) {
  if (std::isnan(v)) {
    std::memcpy(buf, "NaN", 3);
    return 3;
  }
  if (std::isinf(v)) {
    std::memcpy(buf, v > 0 ? "+Inf" : "-Inf", 4);
    return 4;
  }
  // Integral values (bytes, counts, PIDs) print without exponent, like Go's
  // strconv 'g' for <1e21 only when they are short; Prometheus parses either form.
  if (v == std::floor(v) && std::fabs(v) < 9007199254740992.0)
    return size_t(std::to_chars(buf, buf + 40, static_cast<long long>(v)).ptr - buf);
  return size_t(std::to_chars(buf, buf + 40, v).ptr - buf);
}

void append_value(std::string* out, double v) {
  char buf[40];
  out->append(buf, format_value(buf, v));
}

void append_escaped_label_value(std::string* out, const std::string& v) {
  for (char c : v) {
    switch (c) {
      case '\\': out->append("\\\\"); break;
      case '"': out->append("\\\""); break;
      case '\n': out->append("\\n"); break;
      default: out->push_back(c);
    }
  }
}

void append_escaped_help(std::string* out, const std::string& v) {
  for (char c : v) {
    switch (c) {
      case '\\': out->append("\\\\"); break;
      case '\n': out->append("\\n"); break;
      default: out->push_back(c);
    }
  }
}

static bool name_ok(const std::string& s, bool allow_colon) {
  if (s.empty()) return false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    bool alpha = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_' ||
                 (allow_colon && c == ':');
    bool digit = c >= '0' && c <= '9';
    if (!(alpha || (i > 0 && digit))) return false;
  }
  return true;
}

bool valid_metric_name(const std::string& s) { return name_ok(s, true); }
bool valid_label_name(const std::string& s) {
  return name_ok(s, false) && !(s.size() >= 2 && s[0] == '_' && s[1] == '_');
}

int SeriesTable::add_family(const FamilyDef& def) {
  if (!valid_metric_name(def.name)) throw std::invalid_argument("bad metric name: " + def.name);
  for (auto& l : def.label_names)
    if (!valid_label_name(l)) throw std::invalid_argument("bad label name: " + l);
  if (family_id(def.name) >= 0) throw std::invalid_argument("duplicate family: " + def.name);
  Family f;
  f.def = def;
  f.header = "# HELP " + def.name + " ";
  append_escaped_help(&f.header, def.help);
  static const char* tn[] = {"gauge", "counter", "histogram"};
  f.header += "\n# TYPE " + def.name + " " + tn[int(def.type)] + "\n";
  families_.push_back(std::move(f));
  fam_hot_.emplace_back();
  debug_relayout_ = std::getenv("GPUEXP_DEBUG_RELAYOUT") != nullptr;
  int fid = int(families_.size() - 1);
  render_order_.push_back(fid);
  std::sort(render_order_.begin(), render_order_.end(), [this](int a, int b) {
    return families_[size_t(a)].def.name < families_[size_t(b)].def.name;
  });
  return fid;
}

int SeriesTable::family_id(const std::string& name) const {
  for (size_t i = 0; i < families_.size(); ++i)
    if (families_[i].def.name == name) return int(i);
  return -1;
}

SeriesRef SeriesTable::upsert(int fid, const std::vector<std::string>& values) {
  Family& fam = families_.at(size_t(fid));
  if (values.size() != fam.def.label_names.size())
    throw std::invalid_argument("label arity mismatch for " + fam.def.name);
  keybuf_.clear();
  keybuf_.append(reinterpret_cast<const char*>(&fid), sizeof(fid));
  for (auto& v : values) {
    keybuf_.append(v);
    keybuf_.push_back('\0');
  }
  auto it = index_.find(keybuf_);
  if (it != index_.end()) return SeriesRef{it->second, hot_[it->second].ver};

  uint32_t idx;
  if (!free_.empty()) {
    idx = free_.back();
    free_.pop_back();
  } else {
    idx = uint32_t(series_.size());
    series_.emplace_back();
    hot_.emplace_back();
  }
  Hot& h = hot_[idx];
  Series& s = series_[idx];
  h.fid = fid;
  h.ver += 1;
  h.gen = 0;
  h.value = 0;
  h.in_cache = false;
  h.laid = false;
  h.stamp += 1;
  s.widths.clear();
  s.labels = values;
  s.key = keybuf_;
  s.bounds.clear();
  s.buckets.clear();
  s.hsum = 0;
  s.hcount = 0;
  s.prefix = fam.def.name;
  if (!values.empty()) {
    s.prefix.push_back('{');
    for (size_t i = 0; i < values.size(); ++i) {
      if (i) s.prefix.push_back(',');
      s.prefix.append(fam.def.label_names[i]);
      s.prefix.append("=\"");
      append_escaped_label_value(&s.prefix, values[i]);
      s.prefix.push_back('"');
    }
    s.prefix.push_back('}');
  }
  s.line = s.prefix;
  s.line.push_back(' ');
  s.vvalid = false;
  s.hlines.clear();
  index_.emplace(s.key, idx);
  fam.members.push_back(idx);
  FamHot& fh = fam_hot_[size_t(fid)];
  fh.nmembers += 1;
  fh.dirty_order = true;
  fh.dirty = true;
  return SeriesRef{idx, h.ver};
}

bool SeriesTable::set(SeriesRef r, double v, uint64_t gen) {
  if (!r.valid() || r.idx >= hot_.size()) return false;
  Hot& h = hot_[r.idx];
  if (h.ver != r.ver || h.fid < 0) return false;
  uint64_t a, b;
  std::memcpy(&a, &h.value, sizeof(a));
  std::memcpy(&b, &v, sizeof(b));
  if (a != b) h.value = v;
  note_set(h, gen, a != b);
  return true;
}

bool SeriesTable::touch(SeriesRef r, uint64_t gen) {
  if (!r.valid() || r.idx >= hot_.size()) return false;
  Hot& h = hot_[r.idx];
  if (h.ver != r.ver || h.fid < 0) return false;
  note_set(h, gen, false);
  return true;
}

bool SeriesTable::observe(SeriesRef r, double v, uint64_t gen, const std::vector<double>& bounds) {
  if (!r.valid() || r.idx >= hot_.size()) return false;
  Hot& h = hot_[r.idx];
  if (h.ver != r.ver || h.fid < 0) return false;
  Series& s = series_[r.idx];
  if (s.bounds.empty()) {
    s.bounds = bounds;
    s.buckets.assign(bounds.size(), 0);
    s.hlines.clear();
  }
  // Buckets are stored non-cumulative; rendering accumulates.
  auto it = std::lower_bound(s.bounds.begin(), s.bounds.end(), v);
  if (it != s.bounds.end()) s.buckets[size_t(it - s.bounds.begin())] += 1;
  s.hsum += v;
  s.hcount += 1;
  note_set(h, gen, true);
  return true;
}

bool SeriesTable::set_histogram(SeriesRef r, const std::vector<double>& bounds,
                                const std::vector<uint64_t>& counts, double sum, uint64_t count,
                                uint64_t gen) {
  if (!r.valid() || r.idx >= hot_.size()) return false;
  Hot& h = hot_[r.idx];
  if (h.ver != r.ver || h.fid < 0) return false;
  Series& s = series_[r.idx];
  bool changed = s.hcount != count || s.hsum != sum || s.bounds != bounds;
  if (s.bounds != bounds) {
    s.bounds = bounds;
    s.hlines.clear();
  }
  s.buckets.resize(bounds.size(), 0);
  for (size_t i = 0; i < bounds.size(); ++i) {
    const uint64_t c = i < counts.size() ? counts[i] : 0;
    changed = changed || s.buckets[i] != c;
    s.buckets[i] = c;
  }
  s.hsum = sum;
  s.hcount = count;
  note_set(h, gen, changed);
  return true;
}

double SeriesTable::value(SeriesRef r) const {
  if (!r.valid() || r.idx >= hot_.size()) return std::nan("");
  const Hot& h = hot_[r.idx];
  if (h.ver != r.ver) return std::nan("");
  return h.value;
}

void SeriesTable::free_series(uint32_t idx) {
  Hot& h = hot_[idx];
  Series& s = series_[idx];
  index_.erase(s.key);
  if (h.fid >= 0) {
    FamHot& f = fam_hot_[size_t(h.fid)];
    f.dirty = true;
    f.nmembers -= 1;
    if (h.laid) f.laid_valid = false;  // (cannot happen while laid: only stale members are freed)
  }
  h.fid = -1;
  h.ver += 1;
  h.in_cache = false;
  h.laid = false;
  h.stamp += 1;
  s.widths.clear();
  s.labels.clear();
  s.prefix.clear();
  s.line.clear();
  s.key.clear();
  s.bounds.clear();
  s.buckets.clear();
  s.hlines.clear();
  s.vvalid = false;
  free_.push_back(idx);
}

void SeriesTable::sort_members(int fid) {
  Family& f = families_[size_t(fid)];
  std::sort(f.members.begin(), f.members.end(), [this](uint32_t a, uint32_t b) {
    const auto& la = series_[a].labels;
    const auto& lb = series_[b].labels;
    for (size_t i = 0; i < la.size(); ++i) {
      if (la[i] != lb[i]) {
        // numeric-aware ordering so gpu="10" sorts after gpu="9"
        bool da = !la[i].empty() && la[i].find_first_not_of("0123456789") == std::string::npos;
        bool db = !lb[i].empty() && lb[i].find_first_not_of("0123456789") == std::string::npos;
        if (da && db && la[i].size() != lb[i].size()) return la[i].size() < lb[i].size();
        return la[i] < lb[i];
      }
    }
    return false;
  });
  fam_hot_[size_t(fid)].dirty_order = false;
  fam_hot_[size_t(fid)].dirty = true;
}

void SeriesTable::unlay(int fid) {
  Layout& L = layouts_[size_t(fid)];
  for (const LaidMember& m : L.members) {
    Hot& h = hot_[m.idx];
    if (h.ver == m.ver && h.fid == fid) h.laid = false;
  }
  fam_hot_[size_t(fid)].laid_valid = false;
  fam_hot_[size_t(fid)].nlaid = 0;
}

void SeriesTable::format_cached(uint32_t idx) {
  Series& s = series_[idx];
  const double v = hot_[idx].value;
  uint64_t bits;
  std::memcpy(&bits, &v, sizeof(bits));
  if (!s.vvalid || bits != s.vbits) {
    char buf[40];
    const size_t n = format_value(buf, v);
    s.vlen = uint8_t(std::min(n, sizeof(s.vtxt)));
    std::memcpy(s.vtxt, buf, s.vlen);
    s.vbits = bits;
    s.vvalid = true;
  }
}

void SeriesTable::append_cached_value(std::string* out, uint32_t idx) {
  format_cached(idx);
  out->append(series_[idx].vtxt, series_[idx].vlen);
}

void SeriesTable::build_hlines(uint32_t idx) {
  Series& s = series_[idx];
  if (s.hlines.size() != s.bounds.size() + 3) {
    const Family& fam = families_[size_t(hot_[idx].fid)];
    const std::string& base = fam.def.name;
    std::string labels;  // `a="x",b="y"`
    if (s.prefix.size() > base.size() + 2) labels = s.prefix.substr(base.size() + 1, s.prefix.size() - base.size() - 2);
    s.hlines.clear();
    for (size_t i = 0; i <= s.bounds.size(); ++i) {
      std::string l = base + "_bucket{";
      if (!labels.empty()) l += labels + ",";
      l += "le=\"";
      if (i < s.bounds.size()) append_value(&l, s.bounds[i]);
      else l += "+Inf";
      l += "\"} ";
      s.hlines.push_back(std::move(l));
    }
    for (const char* sfx : {"_sum", "_count"}) {
      std::string l = base + sfx;
      if (!labels.empty()) l += "{" + labels + "}";
      l += " ";
      s.hlines.push_back(std::move(l));
    }
  }
}

void SeriesTable::render_histogram(std::string* out, uint32_t idx) {
  // name_bucket{labels,le="x"} cumulative ... _sum, _count.  The line prefixes depend only
  // on the labels and the (fixed) bounds: built once, then each render appends numbers.
  build_hlines(idx);
  Series& s = series_[idx];
  char buf[24];
  uint64_t cum = 0;
  for (size_t i = 0; i <= s.bounds.size(); ++i) {
    cum = i < s.bounds.size() ? cum + s.buckets[i] : s.hcount;
    out->append(s.hlines[i]);
    auto r = std::to_chars(buf, buf + sizeof(buf), cum);
    out->append(buf, r.ptr);
    out->push_back('\n');
  }
  out->append(s.hlines[s.bounds.size() + 1]);
  append_value(out, s.hsum);
  out->push_back('\n');
  out->append(s.hlines[s.bounds.size() + 2]);
  auto r = std::to_chars(buf, buf + sizeof(buf), s.hcount);
  out->append(buf, r.ptr);
  out->push_back('\n');
}

void SeriesTable::render(std::string* out, uint64_t gen, uint64_t gc_after) {
  out->clear();
  last_rebuilt_ = 0;
  for (int fid : render_order_) {
    Family& fam = families_[size_t(fid)];
    // GC + liveness pass over the dense hot array: drop members stale for longer than
    // gc_after gens; a member whose liveness differs from the cached text dirties it.
    bool any_live = false;
    size_t w = 0;
    for (size_t i = 0; i < fam.members.size(); ++i) {
      uint32_t idx = fam.members[i];
      Hot& h = hot_[idx];
      if (h.gen + gc_after < gen) {
        free_series(idx);
        continue;
      }
      fam.members[w++] = idx;
      const bool live = h.gen == gen;
      any_live = any_live || live;
      if (live != h.in_cache) fam_hot_[size_t(fid)].dirty = true;
    }
    fam.members.resize(w);
    if (!any_live) {
      if (!fam.cache.empty()) {
        fam.cache.clear();
        for (uint32_t idx : fam.members) hot_[idx].in_cache = false;
      }
      fam_hot_[size_t(fid)].dirty = false;
      continue;
    }
    if (fam_hot_[size_t(fid)].dirty_order) sort_members(fid);
    if (fam_hot_[size_t(fid)].dirty) {
      ++last_rebuilt_;
      fam.cache.clear();
      fam.cache.append(fam.header);
      for (uint32_t idx : fam.members) {
        Hot& h = hot_[idx];
        h.in_cache = h.gen == gen;
        if (!h.in_cache) continue;
        if (fam.def.type == MetricType::kHistogram) {
          render_histogram(&fam.cache, idx);
          continue;
        }
        fam.cache.append(series_[idx].line);
        append_cached_value(&fam.cache, idx);
        fam.cache.push_back('\n');
      }
      fam_hot_[size_t(fid)].dirty = false;
    }
    out->append(fam.cache);
  }
}

void SeriesTable::field_texts(uint32_t idx) {
  const Hot& h = hot_[idx];
  Series& s = series_[idx];
  if (families_[size_t(h.fid)].def.type != MetricType::kHistogram) {
    format_cached(idx);
    scratch_.resize(32);
    scratch_len_.assign(1, s.vlen);
    std::memcpy(scratch_.data(), s.vtxt, s.vlen);
    return;
  }
  const size_t nf = s.bounds.size() + 3;
  scratch_.resize(32 * nf);
  scratch_len_.resize(nf);
  uint64_t cum = 0;
  auto put_u64 = [&](size_t f, uint64_t v) {
    auto r = std::to_chars(&scratch_[32 * f], &scratch_[32 * f] + 32, v);
    scratch_len_[f] = uint8_t(r.ptr - &scratch_[32 * f]);
  };
  for (size_t i = 0; i <= s.bounds.size(); ++i) {
    cum = i < s.bounds.size() ? cum + s.buckets[i] : s.hcount;
    put_u64(i, cum);
  }
  char tmp[40];
  const size_t tn = format_value(tmp, s.hsum);
  const size_t fs = s.bounds.size() + 1;
  scratch_len_[fs] = uint8_t(std::min<size_t>(tn, 32));
  std::memcpy(&scratch_[32 * fs], tmp, scratch_len_[fs]);
  put_u64(fs + 1, s.hcount);
}

void SeriesTable::layout_family(int fid, uint64_t gen, std::string* body) {
  Family& fam = families_[size_t(fid)];
  Layout& L = layouts_[size_t(fid)];
  if (debug_relayout_) std::fprintf(stderr, "[exposition] gen %llu: %s laid out again (%s)\n", (unsigned long long)gen,
                                    fam.def.name.c_str(), L.why);
  unlay(fid);
  L.members.clear();
  L.seg.fields.clear();
  const size_t base = body->size();
  body->append(fam.header);
  const bool hist = fam.def.type == MetricType::kHistogram;
  const std::string& nm = fam.def.name;
  auto ends = [&](const char* suf) {
    const size_t n = std::strlen(suf);
    return nm.size() >= n && nm.compare(nm.size() - n, n, suf) == 0;
  };
  const bool frac_unit = ends("_seconds") || ends("_seconds_total") || ends("_percent") || ends("_ratio") ||
                         ends("_per_second");
  for (uint32_t idx : fam.members) {
    Hot& h = hot_[idx];
    if (h.gen != gen) continue;
    Series& s = series_[idx];
    field_texts(idx);
    const size_t nf = scratch_len_.size();
    if (s.widths.size() != nf) s.widths.assign(nf, 0);
    if (hist) build_hlines(idx);
    L.members.push_back({idx, h.ver, h.stamp, uint32_t(L.seg.fields.size()), gen});
    h.laid = true;
    for (size_t f = 0; f < nf; ++f) {
      body->append(hist ? s.hlines[f] : s.line);
      const uint8_t len = scratch_len_[f];
      // Room to grow, so the body settles within a few ticks (on silicon the first ~10 ticks laid
      // out ~100 families again: sentinel latencies, activity percentages).  A fraction may later
      // print as any shortest round-trip form, up to 24 characters ("-1.2345678901234567e-308"),
      // so it gets all 24 from the start (with 20, each GPU's CPU-seconds counter on a fake 8-GPU
      // node outgrew its field at its own tick, one relayout each); so does a value of a
      // fractional unit still integral (a latency of 0 before its first sample).  An integer gets
      // one more digit (a gauge) or two (a counter or histogram count: they only grow), and two
      // more whenever it outgrows its field.
      if (!s.widths[f] || len > s.widths[f]) {
        const char* t = &scratch_[32 * f];
        const bool frac = std::memchr(t, '.', len) || std::memchr(t, 'e', len) ||
                          (frac_unit && (!hist || f == s.bounds.size() + 1));
        const int room = s.widths[f] || fam.def.type != MetricType::kGauge ? 2 : 1;
        s.widths[f] = uint8_t(frac ? std::max<int>(len, 24) : std::min<int>(32, len + room));
      }
      s.widths[f] = std::max(s.widths[f], len);
      L.seg.fields.push_back({uint32_t(body->size() - base), s.widths[f]});
      // right-aligned: the blanks sit between "} " and the value, where every text parser
      // skips them (client_golang's expfmt reads a blank AFTER a value as a timestamp separator)
      body->append(size_t(s.widths[f] - len), ' ');
      body->append(&scratch_[32 * f], len);
      body->push_back('\n');
    }
  }
  L.seg.base = base;
  L.seg.len = body->size() - base;
  L.seg.parsed = false;
  L.seg.code_epoch = 0;
  L.seg.splice_valid = false;
  L.seg.changed_gen = gen;
  L.seg.layout_ver += 1;
  L.valid = true;
  L.relayout = false;
  FamHot& fh = fam_hot_[size_t(fid)];
  fh.change_gen = gen;
  fh.laid_valid = true;
  fh.nlaid = uint32_t(L.members.size());
  // this generation's counts as the layout sees them (every member laid out is live now)
  fh.live_laid = fh.gen == gen ? uint32_t(L.members.size()) : 0;
}

void SeriesTable::render_compiled(std::string* out, std::string* gz, uint64_t gen, uint64_t gc_after,
                                  uint64_t out_gen) {
  last_rebuilt_ = 0;
  last_relayouts_ = 0;
  last_skipped_ = 0;
  last_walked_ = 0;
  bool rebuild = false;  // some family is laid out again, appears or disappears
  if (layouts_.size() != families_.size()) {
    layouts_.resize(families_.size());  // csegs_ points into layouts_: rebuilt below
    for (size_t f = 0; f < layouts_.size(); ++f) {
      layouts_[f].valid = false;
      fam_hot_[f].laid_valid = false;
    }
    rebuild = true;
  }
  // Families can be passed over by their FamHot counts alone only if every generation since the
  // last pass was rendered (a skipped publish would leave its changes unpatched).
  const bool consecutive = compiled_gen_ && gen == compiled_gen_ + 1;
  compiled_gen_ = gen;
  for (int fid : render_order_) {
    FamHot& fh = fam_hot_[size_t(fid)];
    if (fh.nmembers == 0 && !fh.laid_valid) continue;  // no series (an optional source off): nothing to do
    // unchanged since the last pass: every laid-out member set again, none changed, no other
    // member live or waiting for GC
    if (consecutive && fh.laid_valid && !fh.dirty_order && fh.gen == gen && fh.changed == 0 &&
        fh.live == fh.nlaid && fh.live_laid == fh.nlaid && fh.nmembers == fh.nlaid) {
      ++last_skipped_;
      continue;
    }
    Family& fam = families_[size_t(fid)];
    Layout& L = layouts_[size_t(fid)];
    ++last_walked_;
    if (fh.dirty_order) {  // a new member: laid out again (sorting first, so GC below keeps order)
      sort_members(fid);
      L.relayout = true;
      L.why = "new_series";
    }
    // one pass: GC, liveness, the same live members in the same order as laid out, and the
    // fields of changed members patched in place (a value that outgrew its field, or a
    // membership change, lays the family out again)
    bool any_live = false;
    bool patch = L.valid && !L.relayout;
    size_t w = 0, k = 0;
    const size_t nm = fam.members.size();
    for (size_t i = 0; i < nm; ++i) {
      if (i + 4 < nm) __builtin_prefetch(&hot_[fam.members[i + 4]]);
      const uint32_t idx = fam.members[i];
      const Hot& h = hot_[idx];
      if (h.gen + gc_after < gen) {
        free_series(idx);  // (stale: not in the live sequence compared below)
        continue;
      }
      fam.members[w++] = idx;
      if (h.gen != gen) continue;
      any_live = true;
      if (!patch) continue;
      if (k >= L.members.size() || L.members[k].idx != idx || L.members[k].ver != h.ver) {
        patch = false;
        if (!L.relayout) L.why = "membership";
        continue;
      }
      LaidMember& lm = L.members[k];
      if (h.stamp != lm.stamp) {
        field_texts(idx);
        const size_t nf = scratch_len_.size();
        const TmplField* fl = &L.seg.fields[lm.first_field];
        bool fits = lm.first_field + nf <= L.seg.fields.size();
        for (size_t f = 0; fits && f < nf; ++f) fits = scratch_len_[f] <= fl[f].width;
        if (!fits) {
          patch = false;
          L.why = "outgrown";
          continue;
        }
        for (size_t f = 0; f < nf; ++f) {
          char* dst = &cbody_[L.seg.base + fl[f].off];
          const size_t pad = fl[f].width - scratch_len_[f];
          std::memset(dst, ' ', pad);
          std::memcpy(dst + pad, &scratch_[32 * f], scratch_len_[f]);
        }
        lm.stamp = h.stamp;
        lm.change_gen = gen;
        fh.change_gen = gen;
        L.seg.splice_valid = false;
      }
      ++k;
    }
    fam.members.resize(w);
    if (!any_live) {
      if (L.valid) {
        rebuild = true;
        unlay(fid);
      }
      L.valid = false;
      L.relayout = false;
      continue;
    }
    if (!patch || k != L.members.size()) {
      if (!L.valid) L.why = "appeared";
      else if (patch) L.why = "membership";
      L.relayout = true;
      rebuild = true;
    }
  }
  if (rebuild) {
    parse_check_ = true;  // (checked at the next gzip encode, which may be ticks later)
    rebuild_gen_ = gen;
    cbody_next_.clear();
    csegs_.clear();
    for (int fid : render_order_) {
      Layout& L = layouts_[size_t(fid)];
      if (!L.valid && !L.relayout) continue;
      if (L.relayout) {
        layout_family(fid, gen, &cbody_next_);
        ++last_relayouts_;
        ++last_rebuilt_;
      } else {
        const size_t nb = cbody_next_.size();
        cbody_next_.append(cbody_, L.seg.base, L.seg.len);
        L.seg.base = nb;
      }
      csegs_.push_back(&L.seg);
    }
    cbody_.swap(cbody_next_);
  }
  // Into `out`: the changed fields only, if `out` holds this layout's body as of out_gen.
  if (out_gen && out_gen < gen && out_gen >= rebuild_gen_ && out->size() == cbody_.size()) {
    size_t copied = 0;
    char* o = &(*out)[0];
    for (int fid : render_order_) {
      if (fam_hot_[size_t(fid)].change_gen <= out_gen) continue;
      const Layout& L = layouts_[size_t(fid)];
      if (!L.valid) continue;
      const size_t nm = L.members.size();
      for (size_t m = 0; m < nm; ++m) {
        if (L.members[m].change_gen <= out_gen) continue;
        const size_t f1 = m + 1 < nm ? L.members[m + 1].first_field : L.seg.fields.size();
        for (size_t f = L.members[m].first_field; f < f1; ++f) {
          const TmplField& tf = L.seg.fields[f];
          std::memcpy(o + L.seg.base + tf.off, cbody_.data() + L.seg.base + tf.off, tf.width);
          copied += tf.width;
        }
      }
    }
    last_copied_ = copied;
  } else {
    out->assign(cbody_);
    last_copied_ = cbody_.size();
  }
  if (!gz) return;
  // A segment laid out again (and any whose matches reached into it) is first parsed on its own
  // -- matches within its own bytes only, so no other segment's moves can invalidate it and it
  // invalidates none -- while its layout still moves (warm-up: values reaching their widths; a
  // process appearing); once it held for kStableRenders renders it gets one real parse, reaching
  // back into the segments before it (consecutive ones as one run).
  if (parse_check_) {
    // Per segment: one laid out within the last kStableRenders renders is still settling.  A run
    // of settled segments that need a parse gets one, its matches reaching back no further than
    // the nearest settling segment (so a neighbour that moves again cannot invalidate it).
    // A segment parsed with its lookback cut short by a settling neighbour is parsed again once
    // no segment within its window settles any more.
    auto settling = [&](size_t k) { return gen - csegs_[k]->changed_gen < kStableRenders; };
    auto blocked = [&](size_t k) {  // a settling segment within kLookback before segs[k]
      for (size_t m = k; m > 0 && csegs_[k]->base - (csegs_[m - 1]->base + csegs_[m - 1]->len) < kLookback; --m)
        if (settling(m - 1)) return true;
      return false;
    };
    bool pending = false;
    auto needs = [&](size_t k) {
      const TmplSegment* s = csegs_[k];
      if (!TemplateDeflate::parse_valid(csegs_, k) || s->provisional) return true;
      if (!s->capped) return false;
      if (!blocked(k)) return true;
      pending = true;
      return false;
    };
    for (size_t i = 0; i < csegs_.size();) {
      if (!needs(i)) {
        ++i;
        continue;
      }
      if (settling(i)) {
        if (!TemplateDeflate::parse_valid(csegs_, i)) {
          TemplateDeflate::parse(cbody_.data(), csegs_, i, i + 1, 0);
          csegs_[i]->provisional = true;
          ++provisional_parses_;
        }
        pending = true;
        ++i;
        continue;
      }
      size_t j = i;
      for (; j < csegs_.size() && needs(j) && !settling(j); ++j) {
        const TmplSegment* s = csegs_[j];
        // (a capped segment parsed again with its full lookback barely moves the code's statistics)
        if (!s->capped || s->provisional || !TemplateDeflate::parse_valid(csegs_, j)) relaid_bytes_ += s->len;
      }
      size_t lookback = kLookback;
      for (size_t k = i; k > 0; --k) {  // back to the nearest settling segment, at most kLookback
        if (csegs_[i]->base - csegs_[k - 1]->base > kLookback) break;
        if (settling(k - 1)) {
          lookback = csegs_[i]->base - (csegs_[k - 1]->base + csegs_[k - 1]->len);
          break;
        }
      }
      TemplateDeflate::parse(cbody_.data(), csegs_, i, j, lookback);
      if (lookback < kLookback && csegs_[i]->base > lookback)
        for (size_t k = i; k < j && csegs_[k]->base - csegs_[i]->base + lookback < kLookback; ++k)
          csegs_[k]->capped = true;
      i = j;
    }
    parse_check_ = pending;
  }
  // The code is complete (any segment encodes under it); it is rebuilt for compression once half
  // as many bytes as the body holds were (re-)parsed since the last build (a build re-encodes
  // every segment: ~0.7 ms for an 8-GPU body) -- so the first real parse of the whole body, after
  // the warm-up's provisional parses, gets a code of its own.
  if (!deflate_.have_code() || 2 * relaid_bytes_ > cbody_.size()) {
    deflate_.build_code(cbody_.data(), csegs_);
    relaid_bytes_ = 0;
    ++code_builds_;
  }
  deflate_.encode_gzip(cbody_.data(), cbody_.size(), crc32_fast(0, cbody_.data(), cbody_.size()), csegs_, gz);
}

size_t SeriesTable::live_series(uint64_t gen) const {
  size_t n = 0;
  for (auto& h : hot_)
    if (h.fid >= 0 && h.gen == gen) ++n;
  return n;
}

size_t SeriesTable::live_series_in_family(int fid, uint64_t gen) const {
  size_t n = 0;
  for (uint32_t idx : families_[size_t(fid)].members)
    if (hot_[idx].gen == gen) ++n;
  return n;
}

namespace {

// Minimal protobuf wire encoding (proto3) for metrics.proto.
void pb_varint(std::string* out, uint64_t v) {
  while (v >= 0x80) {
    out->push_back(char(uint8_t(v) | 0x80));
    v >>= 7;
  }
  out->push_back(char(v));
}
void pb_tag(std::string* out, int field, int wire) { pb_varint(out, (uint64_t(field) << 3) | uint64_t(wire)); }
void pb_bytes(std::string* out, int field, const std::string& s) {
  pb_tag(out, field, 2);
  pb_varint(out, s.size());
  out->append(s);
}
void pb_double(std::string* out, int field, double v) {
  pb_tag(out, field, 1);
  char b[8];
  std::memcpy(b, &v, 8);
  out->append(b, 8);
}
void pb_u64(std::string* out, int field, uint64_t v) {
  pb_tag(out, field, 0);
  pb_varint(out, v);
}
void pb_msg(std::string* out, int field, const std::string& body) { pb_bytes(out, field, body); }

}  // namespace

void SeriesTable::render_proto(std::string* out, uint64_t gen) const {
  // metrics.proto: MetricFamily{1 name, 2 help, 3 type, 4 metric}; Metric{1 label, 2 gauge,
  // 3 counter, 7 histogram}; LabelPair{1 name, 2 value}; Gauge/Counter{1 value};
  // Histogram{1 sample_count, 2 sample_sum, 3 bucket}; Bucket{1 cumulative_count,
  // 2 upper_bound}.  MetricType: COUNTER 0, GAUGE 1, HISTOGRAM 4.  Like client_golang,
  // label pairs are sorted by name and the +Inf bucket is implicit (sample_count).
  out->clear();
  std::string fam_buf, metric, sub, lp;
  std::vector<size_t> order;
  for (int fid : render_order_) {
    const Family& fam = families_[size_t(fid)];
    bool any = false;
    for (uint32_t idx : fam.members)
      if (hot_[idx].gen == gen) {
        any = true;
        break;
      }
    if (!any) continue;
    const auto& names = fam.def.label_names;
    order.resize(names.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return names[a] < names[b]; });
    fam_buf.clear();
    pb_bytes(&fam_buf, 1, fam.def.name);
    pb_bytes(&fam_buf, 2, fam.def.help);
    const int type = fam.def.type == MetricType::kCounter ? 0 : fam.def.type == MetricType::kGauge ? 1 : 4;
    pb_u64(&fam_buf, 3, uint64_t(type));
    for (uint32_t idx : fam.members) {
      const Series& s = series_[idx];
      if (hot_[idx].gen != gen) continue;
      metric.clear();
      for (size_t i : order) {
        lp.clear();
        pb_bytes(&lp, 1, names[i]);
        pb_bytes(&lp, 2, i < s.labels.size() ? s.labels[i] : std::string());
        pb_msg(&metric, 1, lp);
      }
      sub.clear();
      if (fam.def.type == MetricType::kHistogram) {
        pb_u64(&sub, 1, s.hcount);
        pb_double(&sub, 2, s.hsum);
        uint64_t cum = 0;
        for (size_t b = 0; b < s.bounds.size(); ++b) {
          cum += s.buckets[b];
          lp.clear();
          pb_u64(&lp, 1, cum);
          pb_double(&lp, 2, s.bounds[b]);
          pb_msg(&sub, 3, lp);
        }
        pb_msg(&metric, 7, sub);
      } else {
        pb_double(&sub, 1, hot_[idx].value);
        pb_msg(&metric, fam.def.type == MetricType::kCounter ? 3 : 2, sub);
      }
      pb_msg(&fam_buf, 4, metric);
    }
    pb_varint(out, fam_buf.size());
    out->append(fam_buf);
  }
}

}  // namespace gpuexp
