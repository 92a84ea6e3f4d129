// Probe: what does one HSA queue cost in host memory on MI355X, and why?
// Creates queues one at a time and reports, after each step: VmRSS, the KFD queues of this
// process (/sys/class/kfd/kfd/proc/<pid>/queues/*), and every new mapping of >= 1 MiB in
// /proc/self/smaps with its resident size.  Build: g++ -O1 probe_queue_mem.cc -I/opt/rocm/include
//   -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib -o probe_queue_mem
#include <dirent.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Map {
  std::string range, name;
  long size_kb = 0, rss_kb = 0;
};

std::map<std::string, Map> smaps() {
  std::map<std::string, Map> out;
  std::ifstream f("/proc/self/smaps");
  std::string line;
  Map cur;
  bool have = false;
  while (std::getline(f, line)) {
    if (!line.empty() && std::isxdigit(static_cast<unsigned char>(line[0])) && line.find('-') != std::string::npos &&
        line.find(' ') > line.find('-')) {
      if (have) out[cur.range] = cur;
      cur = Map();
      std::istringstream is(line);
      std::string perms, off, dev, ino;
      is >> cur.range >> perms >> off >> dev >> ino;
      std::getline(is, cur.name);
      have = true;
    } else if (line.compare(0, 5, "Size:") == 0) {
      cur.size_kb = std::atol(line.c_str() + 5);
    } else if (line.compare(0, 4, "Rss:") == 0) {
      cur.rss_kb = std::atol(line.c_str() + 4);
    }
  }
  if (have) out[cur.range] = cur;
  return out;
}

long vmrss_kb() {
  std::ifstream f("/proc/self/status");
  std::string line;
  while (std::getline(f, line))
    if (line.compare(0, 6, "VmRSS:") == 0) return std::atol(line.c_str() + 6);
  return -1;
}

// KFD names its per-process directories by HOST pid, which a process in a PID namespace
// (the gpurun box) does not know: list the queues of every KFD process (on a dedicated box
// that is this probe, plus whatever else holds a KFD context).
uint32_t g_gpuid = 0;  // our agent's KFD gpu_id: other tenants' GPUs on the host are skipped

void kfd_queues() {
  const std::string base = "/sys/class/kfd/kfd/proc";
  DIR* procs = opendir(base.c_str());
  if (!procs) {
    std::printf("  kfd: %s not readable\n", base.c_str());
    return;
  }
  while (dirent* p = readdir(procs)) {
    if (p->d_name[0] == '.') continue;
    const std::string d = base + "/" + p->d_name + "/queues";
    DIR* dir = opendir(d.c_str());
    if (!dir) {
      std::printf("  kfd proc %s: queues not readable\n", p->d_name);
      continue;
    }
    int n = 0;
    while (dirent* e = readdir(dir)) {
      if (e->d_name[0] == '.') continue;
      std::string info, gid;
      for (const char* f : {"type", "size", "gpuid"}) {
        std::ifstream in(d + "/" + e->d_name + "/" + f);
        std::string v;
        std::getline(in, v);
        info += std::string(" ") + f + "=" + v;
        if (std::string(f) == "gpuid") gid = v;
      }
      if (g_gpuid && gid != std::to_string(g_gpuid)) continue;
      ++n;
      std::printf("  kfd proc %s queue %s:%s\n", p->d_name, e->d_name, info.c_str());
    }
    closedir(dir);
    if (n) std::printf("  kfd proc %s queues on our GPU: %d\n", p->d_name, n);
  }
  closedir(procs);
}

std::map<std::string, Map> g_prev;

void report(const char* step) {
  auto now = smaps();
  std::printf("== %s: VmRSS %ld MiB\n", step, vmrss_kb() / 1024);
  for (auto& kv : now) {
    if (g_prev.count(kv.first)) continue;
    if (kv.second.size_kb < 1024) continue;
    std::printf("  new mapping %s size %ld MiB rss %ld MiB %s\n", kv.first.c_str(), kv.second.size_kb / 1024,
                kv.second.rss_kb / 1024, kv.second.name.c_str());
  }
  kfd_queues();
  g_prev = now;
}

hsa_status_t find_gpu(hsa_agent_t a, void* ud) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) {
    *static_cast<hsa_agent_t*>(ud) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

int main(int argc, char** argv) {
  const int nq = argc > 1 ? std::atoi(argv[1]) : 2;
  g_prev = smaps();
  std::printf("== start: VmRSS %ld MiB\n", vmrss_kb() / 1024);
  if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
  report("hsa_init");
  hsa_agent_t gpu{};
  hsa_iterate_agents(find_gpu, &gpu);
  hsa_agent_get_info(gpu, hsa_agent_info_t(HSA_AMD_AGENT_INFO_DRIVER_UID), &g_gpuid);
  std::printf("== our GPU: KFD gpu_id %u\n", g_gpuid);
  // optional: load a code object before any queue exists (does the loader make the queue?)
  if (argc > 2) {
    hsa_code_object_reader_t reader{};
    hsa_executable_t exe{};
    FILE* f = std::fopen(argv[2], "rb");
    std::vector<char> blob;
    if (f) {
      char buf[65536];
      size_t n;
      while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) blob.insert(blob.end(), buf, buf + n);
      std::fclose(f);
    }
    bool ok = !blob.empty() &&
              hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &reader) == HSA_STATUS_SUCCESS &&
              hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe) ==
                  HSA_STATUS_SUCCESS &&
              hsa_executable_load_agent_code_object(exe, gpu, reader, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
              hsa_executable_freeze(exe, nullptr) == HSA_STATUS_SUCCESS;
    report(ok ? "code object loaded + frozen (no queue yet)" : "code object load FAILED");
  }
  std::vector<hsa_queue_t*> qs;
  // GPUEXP_PROBE_SEG=0: queues asking for no private / group segment (the exporter's packets need
  // none: PM4 reads and a scratch-free sentinel) instead of the maximum
  const char* seg_env = std::getenv("GPUEXP_PROBE_SEG");
  const uint32_t seg = seg_env && std::strcmp(seg_env, "0") == 0 ? 0 : UINT32_MAX;
  std::printf("== queue private/group segment size: %s\n", seg ? "UINT32_MAX" : "0");
  for (int i = 0; i < nq; ++i) {
    hsa_queue_t* q = nullptr;
    if (hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, seg, seg, &q) !=
        HSA_STATUS_SUCCESS)
      return 2;
    qs.push_back(q);
    char step[64];
    std::snprintf(step, sizeof(step), "hsa_queue_create #%d (64 slots)", i + 1);
    report(step);
  }
  for (auto* q : qs) hsa_queue_destroy(q);
  report("queues destroyed");
  hsa_shut_down();
  report("hsa_shut_down");
  return 0;
}
