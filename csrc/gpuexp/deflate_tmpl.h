// gzip of an exposition whose layout is fixed and only value fields change between ticks.
//
// Reference counterpart: promhttp compresses the whole rendered body on every scrape
// (/root/reference/main.go:68-70 via client_golang's gzip writer).  A 100 Hz exporter cannot
// afford that (libdeflate level 1: ~86 us for the 47 KB 1-GPU body on MI355X hosts, ~190 us for
// 8 GPUs, every tick).  Here the body is a set of segments (one per metric family) whose static
// bytes -- HELP/TYPE lines, `name{labels} ` prefixes -- stay put between layouts because every
// value lives in a fixed-width field, right-aligned behind leading blanks (every text parser
// skips blanks between the labels and the value; client_golang's expfmt would read blanks after
// a value as a timestamp separator).  So the LZ77 parse of the static bytes (matches never read or cover a field byte) is
// computed once per layout, and so is the Huffman code and the static bits it encodes to.  A tick
// then only splices pre-encoded static bit strings with the field bytes coded as literals (one
// table lookup per character; a padding run is one literal plus one distance-1 match).
//
// Output: one gzip member with one dynamic-Huffman deflate block (RFC 1951 §3.2.7; RFC 1952),
// readable by any inflater.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace gpuexp {

struct TmplField {
  uint32_t off = 0;    // relative to the segment start
  uint16_t width = 0;  // leading blanks + value bytes (right-aligned)
};

struct TmplSegment {
  // Set by the owner whenever the layout changes (then call TemplateDeflate::parse).
  size_t base = 0;  // offset of the segment in the body
  size_t len = 0;
  std::vector<TmplField> fields;  // ascending, non-overlapping, inside [0, len)

  uint64_t layout_ver = 0;  // bumped by the owner on every layout change of this segment
  uint64_t changed_gen = 0; // the owner's generation of that change (how long it has held)

  // Compiled (owned by TemplateDeflate).
  struct Tok {
    uint32_t kind : 2;   // 0 literal run, 1 match, 2 field
    uint32_t len : 30;   // literal count or match length
    uint32_t a;          // literal start (relative), match distance, or field index
  };
  std::vector<Tok> toks;
  // Static bits under the current code: piece i = words[bit_start/64 ...] nbits, then field i
  // (the last piece has no field).  Re-encoded whenever the code changes.
  std::vector<uint64_t> words;
  std::vector<uint32_t> piece_bits;  // nbits of each piece (fields.size() + 1 pieces)
  uint64_t code_epoch = 0;           // epoch of the code `words` were encoded with
  size_t static_bits = 0;            // sum of piece_bits
  size_t field_bytes = 0;            // sum of field widths
  // The segment's whole bit string (static pieces + the fields' bytes as they stand), kept
  // between encodes: the owner clears splice_valid when it patches a field; parse and a new
  // code clear it too.  An unchanged segment is then one spliced copy per encode.
  std::vector<uint64_t> spliced;
  size_t spliced_bits = 0;
  bool splice_valid = false;
  bool parsed = false;
  bool provisional = false;   // parsed on its own (lookback 0, owner's policy): valid, but worth a real parse
  bool capped = false;        // parsed with a short lookback (owner's policy): worth a re-parse later
  // Matches may reach back into preceding segments' static bytes: the parse is valid while the
  // same segments, at the same layout versions, precede this one (nearest first).
  std::vector<std::pair<const TmplSegment*, uint64_t>> deps;
};

class TemplateDeflate {
 public:
  // LZ77 parse of the static bytes of segs[i0, i1) (hash chains with one-step lazy matching).
  // A segment's matches reach up to `lookback` bytes back into the segments before it (their
  // static bytes only); segs tile `body`.  A run of consecutive segments shares one hash state.
  static void parse(const char* body, const std::vector<TmplSegment*>& segs, size_t i0, size_t i1,
                    size_t lookback = 8192);
  // Whether segs[i]'s parse still holds (its cross-segment references point at the same bytes).
  static bool parse_valid(const std::vector<TmplSegment*>& segs, size_t i);

  // Builds the Huffman code from every segment's tokens plus the field bytes currently in
  // `body`, so the static bits and today's values both code short; every character a field can
  // hold stays encodable.  Invalidates every segment's static bits (re-encoded lazily).
  void build_code(const char* body, const std::vector<TmplSegment*>& segs);
  bool have_code() const { return code_epoch_ != 0; }
  uint64_t code_epoch() const { return code_epoch_; }

  // Appends the gzip member for `body` (length `body_len`, CRC-32 `crc`).  Segments must tile
  // the body in order (seg[i].base + len == seg[i+1].base; any bytes between segments and after
  // the last one are coded as literals).
  void encode_gzip(const char* body, size_t body_len, uint32_t crc, const std::vector<TmplSegment*>& segs,
                   std::string* out);

  // Bits of the last encode, for tests/diagnostics.
  size_t last_static_bits() const { return last_static_bits_; }
  size_t last_field_bits() const { return last_field_bits_; }

 private:
  void encode_static(const char* body, TmplSegment* seg) const;
  void splice(const char* body, TmplSegment* seg) const;
  struct Code {
    uint16_t code = 0;  // bit-reversed (deflate writes Huffman codes MSB-first into an LSB-first stream)
    uint8_t len = 0;
  };
  Code lit_[288];
  Code dist_[30];
  std::vector<uint64_t> hdr_words_;  // block header (BFINAL, BTYPE, tables)
  size_t hdr_bits_ = 0;
  uint64_t code_epoch_ = 0;
  // pad[n]: n blanks coded (a literal blank, then a distance-1 match for n >= 4)
  std::vector<uint64_t> pad_bits_;
  std::vector<uint8_t> pad_len_;
  size_t last_static_bits_ = 0, last_field_bits_ = 0;
};

// CRC-32 (gzip's) with libdeflate's folded implementation when present, else zlib's.
uint32_t crc32_fast(uint32_t crc, const void* p, size_t n);

}  // namespace gpuexp
