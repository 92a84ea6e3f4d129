#include <zlib.h>

#include "gpuexp/snapshot.h"

namespace gpuexp {

namespace {
// One deflate state per compressing thread (the sampler), reset per body instead of
// re-initialised: saves the ~270 KB state allocation every tick.
struct Deflater {
  z_stream zs{};
  int level = -100;
  bool ok = false;
  ~Deflater() {
    if (ok) deflateEnd(&zs);
  }
  bool prepare(int lvl) {
    if (ok && lvl == level) return deflateReset(&zs) == Z_OK;
    if (ok) deflateEnd(&zs);
    zs = z_stream{};
    // windowBits 15 + 16 => gzip wrapper; memLevel 8.
    ok = deflateInit2(&zs, lvl, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) == Z_OK;
    level = lvl;
    return ok;
  }
};
}  // namespace

bool gzip_compress(const std::string& in, std::string* out, int level) {
  thread_local Deflater d;
  if (!d.prepare(level)) return false;
  z_stream& zs = d.zs;
  out->resize(deflateBound(&zs, uLong(in.size())) + 32);
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = uInt(in.size());
  zs.next_out = reinterpret_cast<Bytef*>(&(*out)[0]);
  zs.avail_out = uInt(out->size());
  if (deflate(&zs, Z_FINISH) != Z_STREAM_END) {
    d.ok = false;
    deflateEnd(&zs);
    out->clear();
    return false;
  }
  out->resize(zs.total_out);
  return true;
}

}  // namespace gpuexp
