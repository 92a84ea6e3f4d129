// Replays fuzz inputs (files, or every file of a directory) through LLVMFuzzerTestOneInput in a
// build without libFuzzer: g++ -fsanitize=address,undefined with ASan's global redzones on.
// tests/test_sanitizers.py runs the libFuzzer build of the same target for a minute and then
// replays everything it kept -- the checked-in seeds plus the new coverage -- through this one,
// since ROCm clang's coverage instrumentation misplaces instrumented globals and its libFuzzer
// build has to leave them out (see test_deflate_template_fuzz).
#include <dirent.h>
#include <sys/stat.h>

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size);

namespace {

int run_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "cannot read %s\n", path.c_str());
    return 1;
  }
  const std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  LLVMFuzzerTestOneInput(buf.data(), buf.size());
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  int inputs = 0, bad = 0;
  for (int a = 1; a < argc; ++a) {
    struct stat st {};
    if (::stat(argv[a], &st) != 0) {
      std::fprintf(stderr, "no such input %s\n", argv[a]);
      return 2;
    }
    if (!S_ISDIR(st.st_mode)) {
      bad += run_file(argv[a]);
      inputs += 1;
      continue;
    }
    DIR* d = ::opendir(argv[a]);
    while (const dirent* e = d ? ::readdir(d) : nullptr) {
      const std::string p = std::string(argv[a]) + "/" + e->d_name;
      if (e->d_name[0] == '.' || ::stat(p.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) continue;
      bad += run_file(p);
      inputs += 1;
    }
    if (d) ::closedir(d);
  }
  std::printf("replayed %d inputs\n", inputs);
  return bad ? 1 : 0;
}
