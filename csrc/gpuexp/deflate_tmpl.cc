#include "gpuexp/deflate_tmpl.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>

namespace gpuexp {

namespace {

// RFC 1951 §3.2.5 length and distance code tables.
constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
// order in which the code-length code lengths are sent (§3.2.7)
constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

constexpr int kMinMatch = 4;  // hashed on 4 bytes: far fewer chain collisions in label-heavy text
constexpr int kMaxMatch = 258;
constexpr uint32_t kWindow = 32768;
constexpr int kChainDepth = 8;
constexpr int kNiceMatch = 48;  // stop searching at a match this long
constexpr int kLazyBelow = 24;  // look one byte ahead only after a shorter match
constexpr int kHashBits = 13;

int len_sym(int len) {  // 257..285
  int i = 28;
  while (kLenBase[i] > len) --i;
  return 257 + i;
}
int dist_sym(uint32_t d) {
  int i = 29;
  while (kDistBase[i] > d) --i;
  return i;
}

// LSB-first bit sink (deflate's bit order) into a buffer sized by the caller: fewer than 32
// bits pending between calls; whole 64-bit words go out with one store.
struct BitWriter {
  unsigned char* p;
  uint64_t acc = 0;
  unsigned n = 0;
  explicit BitWriter(unsigned char* o) : p(o) {}
  inline void put(uint64_t bits, unsigned k) {  // k <= 32, bits < 2^k
    acc |= bits << n;
    n += k;
    if (n >= 32) {
      const uint32_t w = uint32_t(acc);
      std::memcpy(p, &w, 4);
      p += 4;
      acc >>= 32;
      n -= 32;
    }
  }
  inline void put64(uint64_t w) {
    acc |= w << n;
    std::memcpy(p, &acc, 8);
    p += 8;
    acc = n ? w >> (64 - n) : 0;
  }
  void put_words(const uint64_t* w, size_t nbits) {
    size_t i = 0;
    for (; nbits >= 64; nbits -= 64, ++i) put64(w[i]);
    if (nbits > 32) {
      put(w[i] & 0xffffffffu, 32);
      put((w[i] >> 32) & ((uint64_t(1) << (nbits - 32)) - 1), unsigned(nbits - 32));
    } else if (nbits) {
      put(w[i] & ((uint64_t(1) << nbits) - 1), unsigned(nbits));
    }
  }
  void flush_byte() {
    while (n > 0) {
      *p++ = static_cast<unsigned char>(acc & 0xff);
      acc >>= 8;
      n = n > 8 ? n - 8 : 0;
    }
    acc = 0;
  }
};

// Bit sink into a word vector (static pieces, the block header).
struct WordWriter {
  std::vector<uint64_t>* w;
  size_t bits = 0;
  explicit WordWriter(std::vector<uint64_t>* v) : w(v) {}
  inline void put(uint64_t v, int k) {
    if (!k) return;
    const size_t wi = bits >> 6, off = bits & 63;
    if (wi >= w->size()) w->push_back(0);
    (*w)[wi] |= v << off;
    if (off + size_t(k) > 64) w->push_back(v >> (64 - off));
    bits += size_t(k);
  }
};

uint16_t reverse_bits(uint16_t c, int len) {
  uint16_t r = 0;
  for (int i = 0; i < len; ++i) r = uint16_t((r << 1) | ((c >> i) & 1));
  return r;
}

// Huffman code lengths for `freq` (zeros stay unused), at most `limit` bits.  A plain Huffman
// tree; if it is deeper than the limit, the over-long codes are folded into the limit and the
// Kraft sum is repaired by lengthening the shortest-possible codes one at a time (the classic
// count-based fix-up), then lengths go to symbols by descending frequency.
void huffman_lengths(const uint32_t* freq, int n, int limit, uint8_t* len) {
  std::fill(len, len + n, 0);
  std::vector<int> syms;
  for (int i = 0; i < n; ++i)
    if (freq[i]) syms.push_back(i);
  if (syms.empty()) return;
  if (syms.size() == 1) {  // a lone symbol still needs a 1-bit code
    len[syms[0]] = 1;
    return;
  }
  // two-queue Huffman over frequency-sorted leaves
  std::sort(syms.begin(), syms.end(), [&](int a, int b) { return freq[a] < freq[b] || (freq[a] == freq[b] && a < b); });
  const size_t m = syms.size();
  std::vector<uint64_t> w(2 * m);
  std::vector<int> parent(2 * m, -1);
  for (size_t i = 0; i < m; ++i) w[i] = freq[syms[i]];
  size_t leaf = 0, inner = m, next = m;
  auto take = [&]() -> size_t {
    if (leaf < m && (inner >= next || w[leaf] <= w[inner])) return leaf++;
    return inner++;
  };
  for (size_t k = 0; k + 1 < m; ++k) {
    const size_t a = take(), b = take();
    w[next] = w[a] + w[b];
    parent[a] = parent[b] = int(next);
    ++next;
  }
  std::vector<int> depth(2 * m, 0);
  for (size_t i = next - 1; i-- > 0;) depth[i] = depth[size_t(parent[i])] + 1;
  std::vector<int> count(64, 0);
  for (size_t i = 0; i < m; ++i) ++count[size_t(std::min(depth[i], 63))];
  // fold lengths beyond the limit into it, then repair the Kraft sum
  for (int l = limit + 1; l < 64; ++l) {
    count[size_t(limit)] += count[size_t(l)];
    count[size_t(l)] = 0;
  }
  uint64_t kraft = 0;
  for (int l = 1; l <= limit; ++l) kraft += uint64_t(count[size_t(l)]) << (limit - l);
  while (kraft > (uint64_t(1) << limit)) {
    // make one code at the limit shorter-by-split: move a code from the deepest non-full level
    count[size_t(limit)] -= 1;
    for (int l = limit - 1; l > 0; --l)
      if (count[size_t(l)]) {
        count[size_t(l)] -= 1;
        count[size_t(l + 1)] += 2;
        break;
      }
    kraft -= 1;
  }
  // longest codes to the least frequent symbols (syms is ascending by frequency)
  size_t s = 0;
  for (int l = limit; l >= 1; --l)
    for (int k = 0; k < count[size_t(l)]; ++k) len[syms[s++]] = uint8_t(l);
}

void canonical(const uint8_t* len, int n, uint16_t* code) {
  int bl_count[16] = {0};
  for (int i = 0; i < n; ++i) bl_count[len[i]] += len[i] ? 1 : 0;
  int next[16] = {0};
  int c = 0;
  for (int b = 1; b < 16; ++b) {
    c = (c + bl_count[b - 1]) << 1;
    next[b] = c;
  }
  for (int i = 0; i < n; ++i)
    if (len[i]) code[i] = reverse_bits(uint16_t(next[len[i]]++), len[i]);
}

struct Crc {
  uint32_t (*fn)(uint32_t, const void*, size_t) = nullptr;
  Crc() {
    if (void* h = ::dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL))
      fn = reinterpret_cast<uint32_t (*)(uint32_t, const void*, size_t)>(::dlsym(h, "libdeflate_crc32"));
  }
};

}  // namespace

uint32_t crc32_fast(uint32_t crc, const void* p, size_t n) {
  static const Crc c;
  if (c.fn) return c.fn(crc, p, n);
  return uint32_t(::crc32(uLong(crc), reinterpret_cast<const Bytef*>(p), uInt(n)));
}

bool TemplateDeflate::parse_valid(const std::vector<TmplSegment*>& segs, size_t i) {
  const TmplSegment* seg = segs[i];
  if (!seg->parsed) return false;
  size_t j = i;
  for (const auto& d : seg->deps) {
    if (j == 0) return false;
    --j;
    if (segs[j] != d.first || segs[j]->layout_ver != d.second) return false;
  }
  return true;
}

void TemplateDeflate::parse(const char* body, const std::vector<TmplSegment*>& segs, size_t i0, size_t i1,
                            size_t lookback) {
  if (i1 <= i0) return;
  // window [w0, end): lookback bytes before segs[i0], then the run's segments; one hash state
  // for the whole run, so consecutive segments are hashed once (a segment's lookback is the
  // tail of the one before it)
  lookback = std::min<size_t>(lookback, kWindow - kMaxMatch);
  const size_t w0 = segs[i0]->base > lookback ? segs[i0]->base - lookback : 0;
  const size_t end = segs[i1 - 1]->base + segs[i1 - 1]->len;
  const unsigned char* s = reinterpret_cast<const unsigned char*>(body + w0);
  const uint32_t n = uint32_t(end - w0);
  // static_end[p]: where the static run containing p ends (the next field's start, or n); p
  // itself if p is inside a field
  thread_local std::vector<uint32_t> static_end;
  static_end.assign(n, n);
  {
    size_t first = i0;
    while (first > 0 && segs[first - 1]->base + segs[first - 1]->len > w0) --first;
    uint32_t p = 0;
    for (size_t j = first; j < i1; ++j) {
      const TmplSegment* sj = segs[j];
      for (const TmplField& f : sj->fields) {
        const size_t fo = sj->base + f.off, fe = fo + f.width;
        if (fe <= w0) continue;
        const uint32_t a = uint32_t(std::max(fo, w0) - w0), b = uint32_t(fe - w0);
        for (; p < a; ++p) static_end[p] = a;
        for (; p < b; ++p) static_end[p] = p;
      }
    }
    for (; p < n; ++p) static_end[p] = n;
  }
  // hash table sized to the window (a settling family parsed on its own is a few hundred bytes:
  // clearing 2^13 heads for each of ~100 such parses at start-up cost more than the parses)
  int hb = 8;
  while (hb < kHashBits && (uint32_t(1) << hb) < n) ++hb;
  thread_local std::vector<int32_t> head, prev;
  head.assign(size_t(1) << hb, -1);
  prev.resize(n);
  auto hash = [&](uint32_t p) {
    uint32_t v;
    std::memcpy(&v, s + p, 4);
    return (v * 2654435761u) >> (32 - hb);
  };
  auto insert = [&](uint32_t p) {
    if (p + kMinMatch > static_end[p]) return;  // fewer than 4 static bytes: never a source
    const uint32_t h = hash(p);
    prev[p] = head[h];
    head[h] = int32_t(p);
  };
  // common prefix length of s+a and s+b, at most lim (8 bytes at a time)
  auto common = [&](uint32_t a, uint32_t b, uint32_t lim) {
    uint32_t l = 0;
    while (l + 8 <= lim) {
      uint64_t x, y;
      std::memcpy(&x, s + a + l, 8);
      std::memcpy(&y, s + b + l, 8);
      if (x != y) return l + uint32_t(__builtin_ctzll(x ^ y) >> 3);
      l += 8;
    }
    while (l < lim && s[a + l] == s[b + l]) ++l;
    return l;
  };
  const uint32_t start0 = uint32_t(segs[i0]->base - w0);
  for (uint32_t p = 0; p < start0; ++p) insert(p);
  for (size_t i = i0; i < i1; ++i) {
    TmplSegment* seg = segs[i];
    seg->toks.clear();
    seg->words.clear();
    seg->piece_bits.clear();
    seg->deps.clear();
    seg->code_epoch = 0;
    seg->splice_valid = false;
    seg->provisional = false;
    seg->capped = false;
    const uint32_t start = uint32_t(seg->base - w0);
    const uint32_t seg_end = start + uint32_t(seg->len);
    uint32_t min_src = start;
    auto best_at = [&](uint32_t p, uint32_t* dist) -> int {
      const uint32_t lim = std::min<uint32_t>({uint32_t(kMaxMatch), static_end[p] - p, seg_end - p});
      if (lim < uint32_t(kMinMatch)) return 0;
      int best = 0;
      int depth = kChainDepth;
      for (int32_t q = head[hash(p)]; q >= 0 && depth-- > 0; q = prev[size_t(q)]) {
        const uint32_t d = p - uint32_t(q);
        if (d > kWindow) break;
        const uint32_t ql = std::min(lim, static_end[size_t(q)] - uint32_t(q));
        if (int(ql) <= best || s[size_t(q) + size_t(best)] != s[p + size_t(best)]) continue;
        const uint32_t l = common(uint32_t(q), p, ql);
        if (int(l) > best) {  // nearest first: a tie keeps the nearer source (fewer dependencies)
          best = int(l);
          *dist = d;
          if (l == lim || best >= kNiceMatch) break;
        }
      }
      return best >= kMinMatch ? best : 0;
    };
    uint32_t lit_start = 0, lit_n = 0;
    auto flush_lits = [&]() {
      if (lit_n) seg->toks.push_back({0, lit_n, lit_start - start});
      lit_n = 0;
    };
    size_t fi = 0;
    uint32_t p = start;
    while (p < seg_end) {
      if (fi < seg->fields.size() && p == start + seg->fields[fi].off) {
        flush_lits();
        seg->toks.push_back({2, 0, uint32_t(fi)});
        p += seg->fields[fi].width;
        ++fi;
        continue;
      }
      uint32_t d = 0;
      const int l = best_at(p, &d);
      if (l) {
        // one-step lazy: a longer match at p+1 wins over this one
        uint32_t d2 = 0;
        insert(p);
        const int l2 = (l < kLazyBelow && p + 1 < seg_end && static_end[p + 1] > p + 1) ? best_at(p + 1, &d2) : 0;
        if (l2 > l + 1) {
          if (!lit_n) lit_start = p;
          ++lit_n;
          ++p;
          continue;  // p (now p+1) re-searched next iteration
        }
        flush_lits();
        seg->toks.push_back({1, uint32_t(l), d});
        min_src = std::min(min_src, p - d);
        for (uint32_t k = 1; k < uint32_t(l); ++k) insert(p + k);
        p += uint32_t(l);
        continue;
      }
      insert(p);
      if (!lit_n) lit_start = p;
      ++lit_n;
      ++p;
    }
    flush_lits();
    // the preceding segments the matches read from, nearest first
    const size_t src = w0 + min_src;
    for (size_t j = i; j > 0 && src < segs[j - 1]->base + segs[j - 1]->len; --j)
      seg->deps.emplace_back(segs[j - 1], segs[j - 1]->layout_ver);
    seg->parsed = true;
  }
}

void TemplateDeflate::build_code(const char* body, const std::vector<TmplSegment*>& segs) {
  uint32_t lf[288] = {0}, df[30] = {0};
  for (const TmplSegment* seg : segs) {
    const unsigned char* s = reinterpret_cast<const unsigned char*>(body + seg->base);
    for (const auto& t : seg->toks) {
      if (t.kind == 0) {
        for (uint32_t k = 0; k < t.len; ++k) lf[s[t.a + k]] += 1;
      } else if (t.kind == 1) {
        lf[len_sym(int(t.len))] += 1;
        df[dist_sym(t.a)] += 1;
      } else {
        const TmplField& f = seg->fields[t.a];
        uint32_t pad = 0;  // leading blanks (values are right-aligned), then the value
        while (pad < f.width && s[f.off + pad] == ' ') ++pad;
        for (uint32_t k = pad; k < f.width; ++k) lf[s[f.off + k]] += 1;
        if (pad >= 4) {
          lf[' '] += 1;
          lf[len_sym(int(std::min<uint32_t>(pad - 1, kMaxMatch)))] += 1;
          df[0] += 1;
        } else {
          lf[' '] += pad;
        }
      }
    }
  }
  // A complete code: every byte, length and distance stays encodable, so a segment laid out
  // after this code was built (a new series, a wider field) is encoded with it as it stands
  // and the code is rebuilt only when enough of the body changed (SeriesTable).
  for (int i = 0; i <= 285; ++i) lf[i] += 1;
  for (int i = 0; i < 30; ++i) df[i] += 1;
  uint8_t ll[288], dl[30];
  huffman_lengths(lf, 286, 15, ll);
  ll[286] = ll[287] = 0;
  huffman_lengths(df, 30, 15, dl);
  uint16_t lc[288] = {0}, dc[30] = {0};
  canonical(ll, 288, lc);
  canonical(dl, 30, dc);
  for (int i = 0; i < 288; ++i) lit_[i] = {lc[i], ll[i]};
  for (int i = 0; i < 30; ++i) dist_[i] = {dc[i], dl[i]};

  // block header: BFINAL=1, BTYPE=10, HLIT/HDIST/HCLEN, code-length code, run-length coded lengths
  int nlit = 286, ndist = 30;
  while (nlit > 257 && !ll[nlit - 1]) --nlit;
  while (ndist > 1 && !dl[ndist - 1]) --ndist;
  std::vector<uint8_t> lens(ll, ll + nlit);
  lens.insert(lens.end(), dl, dl + ndist);
  struct Rl {
    uint8_t sym, extra, nextra;
  };
  std::vector<Rl> rl;
  for (size_t i = 0; i < lens.size();) {
    const uint8_t v = lens[i];
    size_t run = 1;
    while (i + run < lens.size() && lens[i + run] == v) ++run;
    size_t left = run;
    if (v == 0) {
      while (left >= 11) {
        const size_t k = std::min<size_t>(left, 138);
        rl.push_back({18, uint8_t(k - 11), 7});
        left -= k;
      }
      if (left >= 3) {
        rl.push_back({17, uint8_t(left - 3), 3});
        left = 0;
      }
      while (left--) rl.push_back({0, 0, 0});
    } else {
      rl.push_back({v, 0, 0});
      --left;
      while (left >= 3) {
        const size_t k = std::min<size_t>(left, 6);
        rl.push_back({16, uint8_t(k - 3), 2});
        left -= k;
      }
      while (left--) rl.push_back({v, 0, 0});
    }
    i += run;
  }
  uint32_t cf[19] = {0};
  for (const Rl& r : rl) cf[r.sym] += 1;
  uint8_t cl[19];
  huffman_lengths(cf, 19, 7, cl);
  uint16_t cc[19] = {0};
  canonical(cl, 19, cc);
  int ncl = 19;
  while (ncl > 4 && !cl[kClOrder[ncl - 1]]) --ncl;
  hdr_words_.clear();
  WordWriter hw(&hdr_words_);
  hw.put(1, 1);  // BFINAL
  hw.put(2, 2);  // BTYPE = dynamic
  hw.put(uint64_t(nlit - 257), 5);
  hw.put(uint64_t(ndist - 1), 5);
  hw.put(uint64_t(ncl - 4), 4);
  for (int i = 0; i < ncl; ++i) hw.put(cl[kClOrder[i]], 3);
  for (const Rl& r : rl) {
    hw.put(cc[r.sym], cl[r.sym]);
    if (r.nextra) hw.put(r.extra, r.nextra);
  }
  hdr_bits_ = hw.bits;

  // padding runs of 0..64 blanks, pre-coded
  pad_bits_.assign(65, 0);
  pad_len_.assign(65, 0);
  for (uint32_t k = 1; k <= 64; ++k) {
    uint64_t b = 0;
    int nb = 0;
    auto add = [&](uint64_t v, int l) {
      b |= v << nb;
      nb += l;
    };
    if (k >= 4) {
      add(lit_[' '].code, lit_[' '].len);
      const int ls = len_sym(int(k - 1));
      add(lit_[ls].code, lit_[ls].len);
      add(uint64_t(k - 1 - kLenBase[ls - 257]), kLenExtra[ls - 257]);
      add(dist_[0].code, dist_[0].len);
    } else {
      for (uint32_t j = 0; j < k; ++j) add(lit_[' '].code, lit_[' '].len);
    }
    if (nb > 64) nb = 0;  // cannot happen with 15-bit codes (<= 4 * 15 + 5)
    pad_bits_[k] = b;
    pad_len_[k] = uint8_t(nb);
  }
  ++code_epoch_;
}

void TemplateDeflate::encode_static(const char* body, TmplSegment* seg) const {
  seg->words.clear();
  seg->piece_bits.clear();
  WordWriter w(&seg->words);
  const unsigned char* s = reinterpret_cast<const unsigned char*>(body + seg->base);
  size_t piece_start = 0;
  for (const auto& t : seg->toks) {
    if (t.kind == 0) {
      for (uint32_t k = 0; k < t.len; ++k) {
        const Code& c = lit_[s[t.a + k]];
        w.put(c.code, c.len);
      }
    } else if (t.kind == 1) {
      const int ls = len_sym(int(t.len));
      w.put(lit_[ls].code, lit_[ls].len);
      w.put(t.len - kLenBase[ls - 257], kLenExtra[ls - 257]);
      const int ds = dist_sym(t.a);
      w.put(dist_[ds].code, dist_[ds].len);
      w.put(t.a - kDistBase[ds], kDistExtra[ds]);
    } else {
      // pieces are word-aligned so each can be spliced on its own
      seg->piece_bits.push_back(uint32_t(w.bits - piece_start));
      w.bits = (w.bits + 63) & ~size_t(63);
      if ((w.bits >> 6) > seg->words.size()) seg->words.resize(w.bits >> 6, 0);
      piece_start = w.bits;
    }
  }
  seg->piece_bits.push_back(uint32_t(w.bits - piece_start));
  seg->static_bits = 0;
  for (uint32_t b : seg->piece_bits) seg->static_bits += b;
  seg->field_bytes = 0;
  for (const TmplField& f : seg->fields) seg->field_bytes += f.width;
  seg->code_epoch = code_epoch_;
  seg->splice_valid = false;
}

void TemplateDeflate::splice(const char* body, TmplSegment* seg) const {
  // bound: the static bits, 15 bits per field byte, and room for the writer's 8-byte stores
  seg->spliced.assign((seg->static_bits + 15 * seg->field_bytes) / 64 + 3, 0);
  unsigned char* start = reinterpret_cast<unsigned char*>(seg->spliced.data());
  BitWriter bw(start);
  const uint64_t* w = seg->words.data();
  const unsigned char* s = reinterpret_cast<const unsigned char*>(body) + seg->base;
  const size_t npieces = seg->piece_bits.size();
  for (size_t i = 0; i < npieces; ++i) {
    const size_t nb = seg->piece_bits[i];
    bw.put_words(w, nb);
    w += (nb + 63) >> 6;
    if (i == seg->fields.size()) break;
    const TmplField& f = seg->fields[i];
    const unsigned char* fp = s + f.off;
    uint32_t lead = 0;  // right-aligned: the blank run first, then the value's bytes
    while (lead < f.width && fp[lead] == ' ') ++lead;
    uint32_t pad = lead;
    while (pad > 64) {  // only for absurd widths
      bw.put(pad_bits_[64] & 0xffffffffu, std::min<unsigned>(32, pad_len_[64]));
      if (pad_len_[64] > 32) bw.put(pad_bits_[64] >> 32, pad_len_[64] - 32u);
      pad -= 64;
    }
    if (pad) {
      const unsigned pl = pad_len_[pad];
      if (pl > 32) {
        bw.put(pad_bits_[pad] & 0xffffffffu, 32);
        bw.put(pad_bits_[pad] >> 32, pl - 32);
      } else {
        bw.put(pad_bits_[pad], pl);
      }
    }
    for (uint32_t k = lead; k < f.width; ++k) {
      const Code& c = lit_[fp[k]];
      bw.put(c.code, c.len);
    }
  }
  seg->spliced_bits = size_t(bw.p - start) * 8 + bw.n;
  if (bw.n) std::memcpy(bw.p, &bw.acc, 8);  // the pending bits (the rest of the buffer is zero)
  seg->splice_valid = true;
}

void TemplateDeflate::encode_gzip(const char* body, size_t body_len, uint32_t crc,
                                  const std::vector<TmplSegment*>& segs, std::string* out) {
  static const unsigned char kHdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
  // exact bound: static bits are known, a field byte codes in at most 15 bits, and bytes
  // outside segments (none when they tile the body) likewise
  size_t bound_bits = hdr_bits_ + 15;
  size_t covered = 0;
  for (TmplSegment* seg : segs) {
    if (seg->code_epoch != code_epoch_) encode_static(body, seg);
    bound_bits += seg->static_bits + 15 * seg->field_bytes;
    covered += seg->len;
  }
  bound_bits += 15 * (body_len - std::min(body_len, covered));
  out->resize(10 + bound_bits / 8 + 8 + 16);
  unsigned char* base = reinterpret_cast<unsigned char*>(&(*out)[0]);
  std::memcpy(base, kHdr, 10);
  BitWriter bw(base + 10);
  bw.put_words(hdr_words_.data(), hdr_bits_);
  size_t static_bits = hdr_bits_, field_bits = 0;
  const unsigned char* b = reinterpret_cast<const unsigned char*>(body);
  size_t pos = 0;
  auto literals = [&](size_t from, size_t to) {
    for (size_t i = from; i < to; ++i) {
      const Code& c = lit_[b[i]];
      bw.put(c.code, c.len);
      field_bits += c.len;
    }
  };
  for (TmplSegment* seg : segs) {
    literals(pos, seg->base);  // bytes between segments (none when segments tile the body)
    if (!seg->splice_valid) splice(body, seg);
    bw.put_words(seg->spliced.data(), seg->spliced_bits);
    static_bits += seg->static_bits;
    field_bits += seg->spliced_bits - seg->static_bits;
    pos = seg->base + seg->len;
  }
  literals(pos, body_len);
  bw.put(lit_[256].code, lit_[256].len);
  bw.flush_byte();
  const uint32_t isize = uint32_t(body_len);
  std::memcpy(bw.p, &crc, 4);
  std::memcpy(bw.p + 4, &isize, 4);
  out->resize(size_t(bw.p + 8 - base));
  last_static_bits_ = static_bits;
  last_field_bits_ = field_bits;
}

}  // namespace gpuexp
