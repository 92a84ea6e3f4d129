// Probe: what does amdsmi expose on this MI355X box, and what does each call cost?
// Build: g++ -O2 -std=c++17 -I/opt/rocm/include tools/probe_amdsmi.cc -L/opt/rocm/lib -lamd_smi -Wl,-rpath,/opt/rocm/lib
#include <amd_smi/amdsmi.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define TIMEIT(label, expr)                                                  \
  do {                                                                       \
    double t0 = now_us();                                                    \
    amdsmi_status_t st_ = AMDSMI_STATUS_SUCCESS;                             \
    for (int it_ = 0; it_ < 50; ++it_) st_ = (expr);                         \
    double dt = (now_us() - t0) / 50;                                        \
    const char* s_ = nullptr;                                                \
    amdsmi_status_code_to_string(st_, &s_);                                  \
    printf("  %-34s %9.1f us  status=%d (%s)\n", label, dt, (int)st_, s_ ? s_ : "?"); \
  } while (0)

int main() {
  double t0 = now_us();
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  printf("amdsmi_init status=%d in %.1f us\n", (int)st, now_us() - t0);
  if (st != AMDSMI_STATUS_SUCCESS) return 1;
  uint32_t nsock = 0;
  amdsmi_get_socket_handles(&nsock, nullptr);
  std::vector<amdsmi_socket_handle> socks(nsock);
  amdsmi_get_socket_handles(&nsock, socks.data());
  printf("sockets=%u\n", nsock);
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    amdsmi_get_processor_handles(socks[s], &np, nullptr);
    std::vector<amdsmi_processor_handle> ph(np);
    amdsmi_get_processor_handles(socks[s], &np, ph.data());
    for (uint32_t p = 0; p < np; ++p) {
      auto h = ph[p];
      amdsmi_bdf_t bdf{};
      amdsmi_get_gpu_device_bdf(h, &bdf);
      char uuid[64] = {0};
      unsigned int ul = sizeof(uuid);
      amdsmi_get_gpu_device_uuid(h, &ul, uuid);
      amdsmi_enumeration_info_t en{};
      amdsmi_get_gpu_enumeration_info(h, &en);
      amdsmi_kfd_info_t kfd{};
      amdsmi_get_gpu_kfd_info(h, &kfd);
      printf("socket %u proc %u bdf=%04lx:%02x:%02x.%x uuid=%s render=%u card=%u hsa=%u hip=%u hip_uuid=%s kfd_id=%lu node=%u part=%u\n",
             s, p, (unsigned long)bdf.domain_number, (unsigned)bdf.bus_number,
             (unsigned)bdf.device_number, (unsigned)bdf.function_number, uuid, en.drm_render,
             en.drm_card, en.hsa_id, en.hip_id, en.hip_uuid, (unsigned long)kfd.kfd_id, kfd.node_id,
             kfd.current_partition_id);
      amdsmi_gpu_metrics_t m{};
      TIMEIT("get_gpu_metrics_info", amdsmi_get_gpu_metrics_info(h, &m));
      printf("  hdr size=%u fmt=%u content=%u\n", m.common_header.structure_size,
             m.common_header.format_revision, m.common_header.content_revision);
      printf("  temp edge=%u hotspot=%u mem=%u vrgfx=%u vrsoc=%u vrmem=%u hbm=%u,%u,%u,%u\n",
             m.temperature_edge, m.temperature_hotspot, m.temperature_mem, m.temperature_vrgfx,
             m.temperature_vrsoc, m.temperature_vrmem, m.temperature_hbm[0], m.temperature_hbm[1],
             m.temperature_hbm[2], m.temperature_hbm[3]);
      printf("  act gfx=%u umc=%u mm=%u gfx_acc=%u mem_acc=%u\n", m.average_gfx_activity,
             m.average_umc_activity, m.average_mm_activity, m.gfx_activity_acc, m.mem_activity_acc);
      printf("  power avg=%u cur=%u energy_acc=%lu sysclk=%lu fwts=%lu accum_ctr=%lu\n",
             m.average_socket_power, m.current_socket_power, (unsigned long)m.energy_accumulator,
             (unsigned long)m.system_clock_counter, (unsigned long)m.firmware_timestamp,
             (unsigned long)m.accumulation_counter);
      printf("  clk avg gfx=%u soc=%u uclk=%u cur gfx=%u soc=%u uclk=%u gfxclks=%u,%u,%u,%u,%u,%u,%u,%u\n",
             m.average_gfxclk_frequency, m.average_socclk_frequency, m.average_uclk_frequency,
             m.current_gfxclk, m.current_socclk, m.current_uclk, m.current_gfxclks[0],
             m.current_gfxclks[1], m.current_gfxclks[2], m.current_gfxclks[3], m.current_gfxclks[4],
             m.current_gfxclks[5], m.current_gfxclks[6], m.current_gfxclks[7]);
      printf("  throttle=%u indep=%lu ppt_res=%lu sock_thm=%lu vr_thm=%lu hbm_thm=%lu prochot=%lu\n",
             m.throttle_status, (unsigned long)m.indep_throttle_status,
             (unsigned long)m.ppt_residency_acc, (unsigned long)m.socket_thm_residency_acc,
             (unsigned long)m.vr_thm_residency_acc, (unsigned long)m.hbm_thm_residency_acc,
             (unsigned long)m.prochot_residency_acc);
      printf("  pcie w=%u s=%u bw_acc=%lu bw_inst=%lu replay=%lu xgmi w=%u s=%u vram_max_bw=%lu parts=%u\n",
             m.pcie_link_width, m.pcie_link_speed, (unsigned long)m.pcie_bandwidth_acc,
             (unsigned long)m.pcie_bandwidth_inst, (unsigned long)m.pcie_replay_count_acc,
             m.xgmi_link_width, m.xgmi_link_speed, (unsigned long)m.vram_max_bandwidth,
             m.num_partition);
      for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l)
        printf("  xgmi[%d] rd=%lu wr=%lu status=%u\n", l, (unsigned long)m.xgmi_read_data_acc[l],
               (unsigned long)m.xgmi_write_data_acc[l], m.xgmi_link_status[l]);
      for (int x = 0; x < 1; ++x) {
        printf("  xcp[%d] gfx_busy_inst=", x);
        for (int c = 0; c < AMDSMI_MAX_NUM_XCC; ++c) printf("%u,", m.xcp_stats[x].gfx_busy_inst[c]);
        printf(" gfx_busy_acc=");
        for (int c = 0; c < AMDSMI_MAX_NUM_XCC; ++c)
          printf("%lu,", (unsigned long)m.xcp_stats[x].gfx_busy_acc[c]);
        printf("\n");
      }
      amdsmi_vram_usage_t vu{};
      TIMEIT("get_gpu_vram_usage", amdsmi_get_gpu_vram_usage(h, &vu));
      printf("  vram total=%u MB used=%u MB\n", vu.vram_total, vu.vram_used);
      uint64_t tot = 0, used = 0;
      TIMEIT("get_gpu_memory_total", amdsmi_get_gpu_memory_total(h, AMDSMI_MEM_TYPE_VRAM, &tot));
      TIMEIT("get_gpu_memory_usage", amdsmi_get_gpu_memory_usage(h, AMDSMI_MEM_TYPE_VRAM, &used));
      printf("  vram total=%lu used=%lu bytes\n", (unsigned long)tot, (unsigned long)used);
      amdsmi_engine_usage_t eu{};
      TIMEIT("get_gpu_activity", amdsmi_get_gpu_activity(h, &eu));
      printf("  activity gfx=%u umc=%u mm=%u\n", eu.gfx_activity, eu.umc_activity, eu.mm_activity);
      amdsmi_power_info_t pi{};
      TIMEIT("get_power_info", amdsmi_get_power_info(h, &pi));
      printf("  power cur=%u avg=%u\n", (unsigned)pi.current_socket_power,
             (unsigned)pi.average_socket_power);
      int64_t temp = 0;
      TIMEIT("get_temp_metric(hotspot)",
             amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &temp));
      printf("  temp hotspot=%ld\n", (long)temp);
      amdsmi_link_metrics_t lm{};
      TIMEIT("get_link_metrics", amdsmi_get_link_metrics(h, &lm));
      printf("  links=%u\n", lm.num_links);
      for (uint32_t l = 0; l < lm.num_links && l < 16; ++l)
        printf("   link[%u] bdf=%02x:%02x.%x rate=%u maxbw=%u type=%d rd=%lu wr=%lu\n", l,
               (unsigned)lm.links[l].bdf.bus_number, (unsigned)lm.links[l].bdf.device_number,
               (unsigned)lm.links[l].bdf.function_number, lm.links[l].bit_rate,
               lm.links[l].max_bandwidth, (int)lm.links[l].link_type,
               (unsigned long)lm.links[l].read, (unsigned long)lm.links[l].write);
      uint32_t nproc = 0;
      TIMEIT("get_gpu_process_list(count)", amdsmi_get_gpu_process_list(h, &nproc, nullptr));
      std::vector<amdsmi_proc_info_t> procs(nproc + 4);
      uint32_t cap = procs.size();
      TIMEIT("get_gpu_process_list(full)",
             (cap = procs.size(), amdsmi_get_gpu_process_list(h, &cap, procs.data())));
      printf("  nproc=%u\n", cap);
      for (uint32_t i = 0; i < cap && i < procs.size(); ++i)
        printf("   pid=%u name=%s mem=%lu vram=%lu gfx_ns=%lu cu_occ=%u container=%s\n",
               (unsigned)procs[i].pid, procs[i].name, (unsigned long)procs[i].mem,
               (unsigned long)procs[i].memory_usage.vram_mem,
               (unsigned long)procs[i].engine_usage.gfx, procs[i].cu_occupancy,
               procs[i].container_name);
      uint64_t e = 0, ts = 0;
      float res = 0;
      TIMEIT("get_energy_count", amdsmi_get_energy_count(h, &e, &res, &ts));
      printf("  energy=%lu res=%g ts=%lu\n", (unsigned long)e, res, (unsigned long)ts);
    }
  }
  amdsmi_shut_down();
  return 0;
}
