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

void kfd_queues() {
  const std::string d = "/sys/class/kfd/kfd/proc/" + std::to_string(getpid()) + "/queues";
  DIR* dir = opendir(d.c_str());
  if (!dir) {
    std::printf("  kfd queues: %s not readable\n", d.c_str());
    return;
  }
  int n = 0;
  while (dirent* e = readdir(dir)) {
    if (e->d_name[0] == '.') continue;
    ++n;
    std::string info;
    for (const char* f : {"type", "size", "gpuid"}) {
      std::ifstream in(d + "/" + e->d_name + "/" + f);
      std::string v;
      std::getline(in, v);
      info += std::string(" ") + f + "=" + v;
    }
    std::printf("  kfd queue %s:%s\n", e->d_name, info.c_str());
  }
  closedir(dir);
  std::printf("  kfd queues total: %d\n", n);
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
  std::vector<hsa_queue_t*> qs;
  for (int i = 0; i < nq; ++i) {
    hsa_queue_t* q = nullptr;
    if (hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q) !=
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
