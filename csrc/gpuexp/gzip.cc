#include <dlfcn.h>
#include <zlib.h>

#include <cstdlib>
#include <cstring>

#include "gpuexp/snapshot.h"

namespace gpuexp {

namespace {

// libdeflate (loaded at run time when the node has it; its C API is declared here since
// the image ships the runtime library without headers) compresses the exposition ~1.8x
// faster than zlib at level 1 and a little smaller: 256 vs 459 us for an 8-GPU full
// profile (104 KB).  GPUEXP_GZIP_IMPL=zlib forces zlib.
struct LibDeflate {
  void* (*alloc)(int) = nullptr;
  size_t (*gzip)(void*, const void*, size_t, void*, size_t) = nullptr;
  size_t (*bound)(void*, size_t) = nullptr;
  void (*release)(void*) = nullptr;
  bool ok = false;
  LibDeflate() {
    const char* impl = std::getenv("GPUEXP_GZIP_IMPL");
    if (impl && std::strcmp(impl, "zlib") == 0) return;
    void* h = ::dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = reinterpret_cast<void* (*)(int)>(::dlsym(h, "libdeflate_alloc_compressor"));
    gzip = reinterpret_cast<size_t (*)(void*, const void*, size_t, void*, size_t)>(
        ::dlsym(h, "libdeflate_gzip_compress"));
    bound = reinterpret_cast<size_t (*)(void*, size_t)>(::dlsym(h, "libdeflate_gzip_compress_bound"));
    release = reinterpret_cast<void (*)(void*)>(::dlsym(h, "libdeflate_free_compressor"));
    ok = alloc && gzip && bound && release;
  }
};

const LibDeflate& libdeflate() {
  static const LibDeflate l;
  return l;
}

// One compressor per compressing thread (the sampler), kept across ticks.
struct DeflateCompressor {
  void* c = nullptr;
  int level = -100;
  ~DeflateCompressor() {
    if (c) libdeflate().release(c);
  }
  void* get(int lvl) {
    if (c && lvl == level) return c;
    if (c) libdeflate().release(c);
    c = libdeflate().alloc(lvl < 1 ? 1 : lvl > 12 ? 12 : lvl);
    level = lvl;
    return c;
  }
};

// zlib fallback: one deflate state per compressing thread, reset per body instead of
// re-initialised (saves the ~270 KB state allocation every tick).
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

const char* gzip_impl() { return libdeflate().ok ? "libdeflate" : "zlib"; }

bool gzip_compress(const std::string& in, std::string* out, int level) {
  if (libdeflate().ok) {
    thread_local DeflateCompressor dc;
    if (void* c = dc.get(level)) {
      out->resize(libdeflate().bound(c, in.size()));
      const size_t n = libdeflate().gzip(c, in.data(), in.size(), &(*out)[0], out->size());
      if (n) {
        out->resize(n);
        return true;
      }
    }
  }
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
