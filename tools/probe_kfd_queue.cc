// Probe (VERDICT r05 Next #6): the host-memory floor of one compute queue created straight
// through KFD (libhsakmt, no ROCr), against ROCr's 2 x 173 MiB (our queue + ROCr's internal
// utility queue, profiles/r05/session14/queue_segments.txt).  The queue is created and
// destroyed without any packet or doorbell write.  Reports VmRSS, new >= 1 MiB mappings and
// this GPU's KFD queues after each step.  Build: g++ -O1 probe_kfd_queue.cc -I/opt/rocm/include
//   /opt/rocm/lib/libhsakmt.a -ldrm -ldrm_amdgpu -lnuma -lpthread -o probe_kfd_queue
#include <dirent.h>
#include <hsakmt/hsakmt.h>
#include <unistd.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>

namespace {

struct Map {
  std::string name;
  long size_kb = 0, rss_kb = 0;
};

std::map<std::string, Map> smaps() {
  std::map<std::string, Map> out;
  std::ifstream f("/proc/self/smaps");
  std::string line, range;
  Map cur;
  while (std::getline(f, line)) {
    const size_t dash = line.find('-'), sp = line.find(' ');
    if (!line.empty() && std::isxdigit(static_cast<unsigned char>(line[0])) && dash != std::string::npos && sp > dash) {
      if (!range.empty()) out[range] = cur;
      cur = Map();
      std::istringstream is(line);
      std::string perms, off, dev, ino;
      is >> range >> perms >> off >> dev >> ino;
      std::getline(is, cur.name);
    } else if (line.compare(0, 5, "Size:") == 0) {
      cur.size_kb = std::atol(line.c_str() + 5);
    } else if (line.compare(0, 4, "Rss:") == 0) {
      cur.rss_kb = std::atol(line.c_str() + 4);
    }
  }
  if (!range.empty()) out[range] = cur;
  return out;
}

long vmrss_kb() {
  std::ifstream f("/proc/self/status");
  std::string line;
  while (std::getline(f, line))
    if (line.compare(0, 6, "VmRSS:") == 0) return std::atol(line.c_str() + 6);
  return -1;
}

uint32_t g_gpuid = 0;
std::map<std::string, Map> g_prev;

void kfd_queues() {
  const std::string base = "/sys/class/kfd/kfd/proc";
  DIR* procs = opendir(base.c_str());
  if (!procs) return;
  while (dirent* p = readdir(procs)) {
    if (p->d_name[0] == '.') continue;
    const std::string d = base + "/" + p->d_name + "/queues";
    DIR* dir = opendir(d.c_str());
    if (!dir) continue;
    int n = 0;
    while (dirent* e = readdir(dir)) {
      if (e->d_name[0] == '.') continue;
      std::string info, gid;
      for (const char* f : {"type", "size", "gpuid"}) {
        std::ifstream in(d + "/" + e->d_name + "/" + f);
        std::string v;
        std::getline(in, v);
        info += std::string(" ") + f + "=" + v;
        if (std::strcmp(f, "gpuid") == 0) gid = v;
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

void report(const char* step) {
  auto now = smaps();
  std::printf("== %s: VmRSS %ld MiB\n", step, vmrss_kb() / 1024);
  for (auto& kv : now) {
    if (g_prev.count(kv.first) || kv.second.size_kb < 1024) continue;
    std::printf("  new mapping %s size %ld MiB rss %ld MiB %s\n", kv.first.c_str(), kv.second.size_kb / 1024,
                kv.second.rss_kb / 1024, kv.second.name.c_str());
  }
  kfd_queues();
  g_prev = now;
}

}  // namespace

int main() {
  g_prev = smaps();
  std::printf("== start: VmRSS %ld MiB\n", vmrss_kb() / 1024);
  if (hsaKmtOpenKFD() != HSAKMT_STATUS_SUCCESS) {
    std::printf("hsaKmtOpenKFD failed\n");
    return 1;
  }
  HsaSystemProperties sys{};
  if (hsaKmtAcquireSystemProperties(&sys) != HSAKMT_STATUS_SUCCESS) return 1;
  int node = -1;
  HsaNodeProperties np{};
  for (HSAuint32 n = 0; n < sys.NumNodes; ++n) {
    if (hsaKmtGetNodeProperties(n, &np) == HSAKMT_STATUS_SUCCESS && np.KFDGpuID && np.NumFComputeCores) {
      node = int(n);
      g_gpuid = np.KFDGpuID;
      break;
    }
  }
  if (node < 0) {
    std::printf("no GPU node\n");
    return 1;
  }
  std::printf("== GPU node %d: KFD gpu_id %u, %u XCCs\n", node, g_gpuid, unsigned(np.NumXcc));
  report("hsaKmtOpenKFD + topology");
  // the AQL ring: 64 packets of 64 bytes in host memory the GPU can reach
  HsaMemFlags fl{};
  fl.ui32.HostAccess = 1;
  fl.ui32.NonPaged = 1;
  fl.ui32.ExecuteAccess = 1;
  fl.ui32.AQLQueueMemory = 1;
  void* ring = nullptr;
  const HSAuint64 ring_bytes = 64 * 64;
  if (hsaKmtAllocMemory(0, 4096, fl, &ring) != HSAKMT_STATUS_SUCCESS || !ring) {
    std::printf("ring alloc failed\n");
    return 1;
  }
  std::memset(ring, 0, 4096);
  HSAuint64 gva = 0;
  if (hsaKmtMapMemoryToGPU(ring, 4096, &gva) != HSAKMT_STATUS_SUCCESS) {
    std::printf("ring map failed\n");
    return 1;
  }
  // the queue's read / write dispatch ids and error-reason payload: inputs for an AQL queue
  // (as ROCr passes its amd_queue_t fields), in a second GPU-mapped host page
  void* ctl = nullptr;
  if (hsaKmtAllocMemory(0, 4096, fl, &ctl) != HSAKMT_STATUS_SUCCESS || !ctl) {
    std::printf("control page alloc failed\n");
    return 1;
  }
  std::memset(ctl, 0, 4096);
  HSAuint64 cva = 0;
  if (hsaKmtMapMemoryToGPU(ctl, 4096, &cva) != HSAKMT_STATUS_SUCCESS) {
    std::printf("control page map failed\n");
    return 1;
  }
  report("ring + control page allocated + mapped");
  HsaQueueResource res{};
  res.Queue_read_ptr_aql = static_cast<HSAuint64*>(ctl);
  res.Queue_write_ptr_aql = static_cast<HSAuint64*>(ctl) + 8;  // own 64-byte line
  res.ErrorReason = reinterpret_cast<volatile HSAint64*>(static_cast<HSAuint64*>(ctl) + 16);
  const HSAKMT_STATUS st = hsaKmtCreateQueue(HSAuint32(node), HSA_QUEUE_COMPUTE_AQL, 100, HSA_QUEUE_PRIORITY_NORMAL,
                                             ring, ring_bytes, nullptr, &res);
  std::printf("== hsaKmtCreateQueue: status %d\n", int(st));
  if (st == HSAKMT_STATUS_SUCCESS) {
    report("KFD compute AQL queue created (no packet, no doorbell)");
    hsaKmtDestroyQueue(res.QueueId);
    report("queue destroyed");
  }
  hsaKmtUnmapMemoryToGPU(ctl);
  hsaKmtFreeMemory(ctl, 4096);
  hsaKmtUnmapMemoryToGPU(ring);
  hsaKmtFreeMemory(ring, 4096);
  hsaKmtReleaseSystemProperties();
  hsaKmtCloseKFD();
  report("hsaKmtCloseKFD");
  return st == HSAKMT_STATUS_SUCCESS ? 0 : 3;
}
