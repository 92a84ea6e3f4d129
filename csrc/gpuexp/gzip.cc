#include <zlib.h>

#include "gpuexp/snapshot.h"

namespace gpuexp {

bool gzip_compress(const std::string& in, std::string* out, int level) {
  z_stream zs{};
  // windowBits 15 + 16 => gzip wrapper; memLevel 8.
  if (deflateInit2(&zs, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  out->resize(deflateBound(&zs, uLong(in.size())) + 32);
  zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
  zs.avail_in = uInt(in.size());
  zs.next_out = reinterpret_cast<Bytef*>(&(*out)[0]);
  zs.avail_out = uInt(out->size());
  int rc = deflate(&zs, Z_FINISH);
  if (rc != Z_STREAM_END) {
    deflateEnd(&zs);
    out->clear();
    return false;
  }
  out->resize(zs.total_out);
  deflateEnd(&zs);
  return true;
}

}  // namespace gpuexp
