// pybind11 module `_gpuexp`: the Python control plane drives the C++ data plane through
// this surface.  Python never runs on the sample or scrape path.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstring>
#include <map>

#include "gpuexp/backends.h"
#include "gpuexp/client.h"
#include "gpuexp/counter_model.h"
#include "gpuexp/engine.h"
#include "gpuexp/kfd_events.h"
#include "gpuexp/exposition.h"
#include "gpuexp/gpu_metrics.h"
#include "gpuexp/pmc_agents.h"
#include "gpuexp/pmc_fake.h"
#include "gpuexp/procs.h"
#include "gpuexp/ras.h"
#include "gpuexp/snapshot.h"

namespace py = pybind11;
using namespace gpuexp;


namespace {

py::dict cgroup_dict(const CgroupInfo& c, bool ok) {
  py::dict d;
  d["kube"] = ok && c.kube;
  d["pod_uid"] = c.pod_uid;
  d["container_id"] = c.container_id;
  d["runtime"] = c.runtime;
  d["qos"] = c.qos;
  d["path"] = c.path;
  return d;
}

py::dict device_dict(const DeviceInfo& d) {
  py::dict o;
  o["index"] = d.index;
  o["uuid"] = d.uuid;
  o["bdf"] = d.bdf;
  o["name"] = d.name;
  o["kfd_gpu_id"] = d.kfd_gpu_id;
  o["render_minor"] = d.render_minor;
  o["hip_id"] = d.hip_id;
  o["vram_total"] = d.vram_total;
  o["num_xcc"] = d.num_xcc;
  o["num_cu"] = d.num_cu;
  o["num_xcc"] = d.num_xcc;
  o["partition_id"] = d.partition_id;
  o["dev_node"] = d.dev_node;
  o["queue_enabled"] = d.queue_enabled;
  py::list keys;
  for (const auto& k : device_owner_keys(d)) keys.append(k);
  o["owner_keys"] = keys;
  o["compute_partition"] = d.compute_partition;
  o["memory_partition"] = d.memory_partition;
  py::list peers;
  for (int l = 0; l < kMaxXgmiLinks; ++l) peers.append(d.xgmi_peer_bdf[l]);
  o["xgmi_peers"] = peers;
  return o;
}

py::dict sample_dict(const DeviceSample& s) {
  py::dict o;
  o["ok"] = s.ok;
  o["error"] = s.error;
  o["gfx_activity"] = s.gfx_activity;
  o["umc_activity"] = s.umc_activity;
  o["vram_used"] = s.vram_used;
  o["power_w"] = s.power_w;
  o["energy_acc"] = s.energy_acc;
  o["temp_hotspot"] = s.temp_hotspot;
  o["temp_mem"] = s.temp_mem;
  o["temp_vrsoc"] = s.temp_vrsoc;
  o["clk_gfx"] = s.clk_gfx;
  o["clk_soc"] = s.clk_soc;
  o["clk_mem"] = s.clk_mem;
  o["num_xgmi_links"] = s.num_xgmi_links;
  py::list rd, wr, up;
  for (int l = 0; l < kMaxXgmiLinks; ++l) {
    rd.append(s.xgmi_read_kb[l]);
    wr.append(s.xgmi_write_kb[l]);
    up.append(s.xgmi_link_up[l]);
  }
  o["xgmi_read_kb"] = rd;
  o["xgmi_write_kb"] = wr;
  o["xgmi_link_up"] = up;
  o["pcie_width"] = s.pcie_width;
  o["pcie_speed_gts"] = s.pcie_speed_gts;
  o["pcie_bw_inst"] = s.pcie_bw_inst;
  o["fw_ts_10ns"] = s.fw_ts_10ns;
  o["accumulation_counter"] = s.accumulation_counter;
  o["res_ppt"] = s.res_ppt;
  o["vram_max_bw_gbs"] = s.vram_max_bw_gbs;
  py::list busy, xclk;
  for (int c = 0; c < kMaxXcc; ++c) {
    busy.append(s.gfx_busy_acc[c]);
    xclk.append(s.clk_gfx_xcc[c]);
  }
  o["gfx_busy_acc"] = busy;
  o["clk_gfx_xcc"] = xclk;
  o["energy_valid"] = s.energy_valid;
  o["energy_unit_j"] = s.energy_unit_j;
  o["residency_valid"] = s.residency_valid;
  o["res_prochot"] = s.res_prochot;
  o["res_socket_thm"] = s.res_socket_thm;
  o["res_vr_thm"] = s.res_vr_thm;
  o["res_hbm_thm"] = s.res_hbm_thm;
  o["pcie_bw_acc"] = s.pcie_bw_acc;
  o["pcie_replay"] = s.pcie_replay;
  o["pcie_nak_sent"] = s.pcie_nak_sent;
  o["pcie_nak_rcvd"] = s.pcie_nak_rcvd;
  o["pcie_l0_recov"] = s.pcie_l0_recov;
  o["xgmi_width"] = s.xgmi_width;
  o["xgmi_speed"] = s.xgmi_speed;
  o["num_partition"] = s.num_partition;
  o["temp_edge"] = s.temp_edge;
  o["temp_vrgfx"] = s.temp_vrgfx;
  o["temp_vrmem"] = s.temp_vrmem;
  return o;
}

ProcSample proc_from_dict(const py::dict& d) {
  ProcSample p;
  p.pid = d["pid"].cast<int>();
  p.vram_bytes = d.contains("vram_bytes") ? d["vram_bytes"].cast<double>() : 0.0;
  p.cu_occupancy = d.contains("cu_occupancy") ? d["cu_occupancy"].cast<double>() : kNaN;
  p.sdma_us = d.contains("sdma_us") ? d["sdma_us"].cast<double>() : kNaN;
  p.evicted_ms = d.contains("evicted_ms") ? d["evicted_ms"].cast<double>() : kNaN;
  p.name = d.contains("name") ? d["name"].cast<std::string>() : "";
  return p;
}

}  // namespace

PYBIND11_MODULE(_gpuexp, m) {
  m.doc() = "MI355X per-pod GPU exporter: native telemetry core";

  m.def("mono_ns", &mono_ns);
  m.def("timer_wakeup_cost", [](double hz, int n) {
    uint64_t cpu = 0, late = 0;
    {
      py::gil_scoped_release rel;
      timer_wakeup_cost(uint64_t(1e9 / hz), n, &cpu, &late);
    }
    return py::make_tuple(cpu, late);
  }, py::arg("hz"), py::arg("n"), "(thread CPU ns per wake-up, mean lateness ns) of the sampler's timer wait");
  m.def("counters_round_policy", [](const std::vector<std::pair<double, bool>>& rounds, double budget, double base_s,
                                     double period_s) {
    // (round CPU ns, late) per finished round -> (EWMA ns, minimum interval s) after each
    double ewma = 0, iv = 0;
    std::vector<std::pair<double, double>> out;
    for (const auto& r : rounds) {
      counters_round_policy(r.first, r.second, budget, base_s * 1e9, period_s * 1e9, &ewma, &iv);
      out.emplace_back(ewma, (iv > 0 ? iv : base_s * 1e9) * 1e-9);
    }
    return out;
  }, py::arg("rounds"), py::arg("budget"), py::arg("base_s"), py::arg("period_s"),
     "counters_cpu_budget's policy over a sequence of (round CPU ns, late) rounds");
  m.def("set_log_level", [](int lvl) { set_log_level(static_cast<LogLevel>(lvl)); });
  m.def("set_log_json", [](bool json) { set_log_json(json); });
  m.def("log", [](int lvl, const std::string& component, const std::string& msg) {
    log_msg(static_cast<LogLevel>(lvl), component.c_str(), msg);
  });
  m.def("format_value", [](double v) {
    std::string s;
    append_value(&s, v);
    return s;
  });
  m.def("escape_label_value", [](const std::string& v) {
    std::string s;
    append_escaped_label_value(&s, v);
    return s;
  });
  m.def("gzip_impl", []() { return std::string(gzip_impl()); });
  m.def("xgmi_peers_from_sysfs", [](const std::string& root, const std::string& bdf) {
    std::string peers[gpuexp::kMaxXgmiLinks];
    gpuexp::xgmi_peers_from_sysfs(root, bdf, peers);
    return std::vector<std::string>(std::begin(peers), std::end(peers));
  }, "xGMI link index -> peer BDF from amdgpu's xgmi_port_num files ('' = no link)");
  m.def("parse_bad_pages", [](const std::string& body) -> py::object {
    gpuexp::RasTotals t;
    if (!gpuexp::parse_bad_pages(body, &t)) return py::none();
    return py::make_tuple(int(t.pages_retired), int(t.pages_pending), int(t.pages_unreservable));
  }, "Parses ras/gpu_vram_bad_pages: (retired, pending, unreservable) or None");
  m.def("kfd_events_drain_fds", [](std::vector<int> fds, int rounds) {
    // drains non-blocking fds (pipes standing in for KFD's SMI event fds) `rounds` times
    KfdEventSource src;
    src.adopt_fds(fds);
    std::vector<std::tuple<int, int, int>> all;
    for (int r = 0; r < rounds; ++r) {
      std::vector<KfdEvent> evs;
      src.drain(&evs);
      for (const KfdEvent& e : evs) all.emplace_back(e.dev, e.event, e.pid);
    }
    return all;
  });
  m.def("parse_kfd_event", [](py::bytes b) -> py::object {
    std::string s(b);
    int ev = 0, pid = -1;
    if (!gpuexp::parse_kfd_event(s.data(), s.size(), &ev, &pid)) return py::none();
    return py::make_tuple(gpuexp::kfd_event_name(ev), pid);
  }, "Parses one KFD SMI event message: (event name, pid or -1), None if malformed");
  m.def("gzip", [](py::bytes b, int level) {
    std::string in = b, out;
    if (!gzip_compress(in, &out, level)) throw std::runtime_error("gzip failed");
    return py::bytes(out);
  }, py::arg("data"), py::arg("level") = 1);
  m.def("parse_cgroup_path", [](const std::string& p) {
    CgroupInfo c;
    bool ok = parse_kube_cgroup_path(p, &c);
    return cgroup_dict(c, ok);
  });
  m.def("parse_proc_cgroup", [](const std::string& content) {
    CgroupInfo c;
    bool ok = parse_proc_cgroup(content, &c);
    return cgroup_dict(c, ok);
  });
  m.def("decode_gpu_metrics", [](py::bytes blob) -> py::object {
    std::string b = blob;
    DeviceSample s;
    if (!decode_gpu_metrics_v1_8(b.data(), b.size(), &s)) return py::none();
    s.ok = true;
    return sample_dict(s);
  });
  m.def("decode_gpu_metrics_raw", [](py::bytes blob) -> py::object {
    // Every field of the v1.8 blob as stored, keyed by the amdsmi Python binding's names
    // (amdsmi_get_gpu_metrics_info), for field-by-field parity checks on hardware.
    std::string b = blob;
    if (b.size() < sizeof(GpuMetricsV1_8)) return py::none();
    GpuMetricsV1_8 g;
    std::memcpy(&g, b.data(), sizeof(g));
    if (g.header.format_revision != 1 || g.header.content_revision != 8) return py::none();
    py::dict o;
    o["temperature_hotspot"] = g.temperature_hotspot;
    o["temperature_mem"] = g.temperature_mem;
    o["temperature_vrsoc"] = g.temperature_vrsoc;
    o["current_socket_power"] = g.curr_socket_power;
    o["average_gfx_activity"] = g.average_gfx_activity;
    o["average_umc_activity"] = g.average_umc_activity;
    o["vram_max_bandwidth"] = g.mem_max_bandwidth;
    o["energy_accumulator"] = g.energy_accumulator;
    o["system_clock_counter"] = g.system_clock_counter;
    o["accumulation_counter"] = g.accumulation_counter;
    o["prochot_residency_acc"] = g.prochot_residency_acc;
    o["ppt_residency_acc"] = g.ppt_residency_acc;
    o["socket_thm_residency_acc"] = g.socket_thm_residency_acc;
    o["vr_thm_residency_acc"] = g.vr_thm_residency_acc;
    o["hbm_thm_residency_acc"] = g.hbm_thm_residency_acc;
    o["gfxclk_lock_status"] = g.gfxclk_lock_status;
    o["pcie_link_width"] = g.pcie_link_width;
    o["pcie_link_speed"] = g.pcie_link_speed;
    o["xgmi_link_width"] = g.xgmi_link_width;
    o["xgmi_link_speed"] = g.xgmi_link_speed;
    o["gfx_activity_acc"] = g.gfx_activity_acc;
    o["mem_activity_acc"] = g.mem_activity_acc;
    o["pcie_bandwidth_acc"] = g.pcie_bandwidth_acc;
    o["pcie_bandwidth_inst"] = g.pcie_bandwidth_inst;
    o["pcie_l0_to_recov_count_acc"] = g.pcie_l0_to_recov_count_acc;
    o["pcie_replay_count_acc"] = g.pcie_replay_count_acc;
    o["pcie_replay_rover_count_acc"] = g.pcie_replay_rover_count_acc;
    o["pcie_nak_sent_count_acc"] = g.pcie_nak_sent_count_acc;
    o["pcie_nak_rcvd_count_acc"] = g.pcie_nak_rcvd_count_acc;
    o["firmware_timestamp"] = g.firmware_timestamp;
    o["current_uclk"] = g.current_uclk;
    o["num_partition"] = g.num_partition;
    o["pcie_lc_perf_other_end_recovery"] = g.pcie_lc_perf_other_end_recovery;
    auto l64 = [](const uint64_t* p, int n) {
      py::list l;
      for (int i = 0; i < n; ++i) l.append(p[i]);
      return l;
    };
    auto l16 = [](const uint16_t* p, int n) {
      py::list l;
      for (int i = 0; i < n; ++i) l.append(p[i]);
      return l;
    };
    o["xgmi_read_data_acc"] = l64(g.xgmi_read_data_acc, 8);
    o["xgmi_write_data_acc"] = l64(g.xgmi_write_data_acc, 8);
    o["xgmi_link_status"] = l16(g.xgmi_link_status, 8);
    o["current_gfxclks"] = l16(g.current_gfxclk, 8);
    o["current_socclks"] = l16(g.current_socclk, 4);
    o["current_vclk0s"] = l16(g.current_vclk0, 4);
    o["current_dclk0s"] = l16(g.current_dclk0, 4);
    py::list busy_acc, busy_inst, low_util;
    for (int x = 0; x < 8; ++x) {
      busy_acc.append(l64(g.xcp_stats[x].gfx_busy_acc, 8));
      low_util.append(l64(g.xcp_stats[x].gfx_low_utilization_acc, 8));
      py::list inst;
      for (int i = 0; i < 8; ++i) inst.append(g.xcp_stats[x].gfx_busy_inst[i]);
      busy_inst.append(inst);
    }
    o["xcp_stats.gfx_busy_acc"] = busy_acc;
    o["xcp_stats.gfx_busy_inst"] = busy_inst;
    o["xcp_stats.gfx_low_utilization_acc"] = low_util;
    return o;
  });
  m.def("gpu_metrics_v1_8_size", []() { return sizeof(GpuMetricsV1_8); });
  // The counter plugins' derivations (counter_model.h) on given deltas: {counter name: delta}
  // over `wall` s for a GPU of `simd` SIMDs and `cu` CUs -> (outputs, scope).
  m.def("derive_counters", [](const py::dict& deltas, double wall, uint32_t simd, uint32_t cu, bool privileged) {
    double d[gpuexp_ctr::kNumCtr] = {};
    int inst[gpuexp_ctr::kNumCtr] = {};
    for (auto kv : deltas) {
      const std::string k = py::str(kv.first);
      int slot = -1;
      for (int c = 0; c < gpuexp_ctr::kNumCtr; ++c)
        if (k == gpuexp_ctr::name(c)) slot = c;
      if (slot < 0) throw std::invalid_argument("unknown counter " + k);
      d[slot] = kv.second.cast<double>();
      inst[slot] = 1;
    }
    gpuexp_ctr::Derived a;
    a.simd = simd;
    a.cu = cu;
    a.privileged = privileged;
    gpuexp_ctr::derive(a, d, inst, wall);
    return py::make_tuple(std::vector<double>(a.latest, a.latest + gpuexp_ctr::kNumOut), a.scope);
  });
  m.def("counter_window_action", [](std::vector<double> d, bool first, double wall, int zero_grbm) {
    // aqlprofile continuous counting's per-window decision (counter_model.h window_action):
    // returns ("publish" | "skip" | "rearm", zero_grbm after the window)
    if (d.size() != size_t(gpuexp_ctr::kNumCtr)) throw std::invalid_argument("one delta per counter");
    const auto act = gpuexp_ctr::window_action(d.data(), first, wall, &zero_grbm);
    static const char* kNames[3] = {"publish", "skip", "rearm"};
    return py::make_tuple(kNames[act], zero_grbm);
  }, py::arg("deltas"), py::arg("first"), py::arg("wall"), py::arg("zero_grbm") = 0);
  // Re-arm back-off decision (counter_model.h rearm_on_reset / rearm_due / rearm_done) over a
  // script of (t_ms, event) with event "backwards" | "stopped" | "armed" | "check"; returns the
  // state after each: (waiting, due_ms, backoff_ms, conflicts, due_now).
  m.def("rearm_policy", [](const std::vector<std::pair<double, std::string>>& events, const std::string& mode,
                           double base_ms, double max_ms, double calm_ms) {
    gpuexp_ctr::RearmConfig c;
    c.mode = mode == "off" ? gpuexp_ctr::kRearmOff : mode == "now" ? gpuexp_ctr::kRearmNow : gpuexp_ctr::kRearmBackoff;
    c.base_ns = int64_t(base_ms * 1e6);
    c.max_ns = int64_t(max_ms * 1e6);
    c.calm_ns = int64_t(calm_ms * 1e6);
    gpuexp_ctr::RearmState s;
    py::list out;
    for (auto& ev : events) {
      const int64_t t = int64_t(ev.first * 1e6) + 1;
      if (ev.second == "backwards" || ev.second == "stopped") gpuexp_ctr::rearm_on_reset(s, c, t, ev.second == "backwards");
      else if (ev.second == "armed") gpuexp_ctr::rearm_done(s, t);
      else if (ev.second != "check") throw std::invalid_argument("unknown event " + ev.second);
      out.append(py::make_tuple(s.waiting, (s.due_ns - 1) / 1e6, s.backoff_ns / 1e6, s.conflicts,
                                gpuexp_ctr::rearm_due(s, c, t)));
    }
    return out;
  }, py::arg("events"), py::arg("mode") = "backoff", py::arg("base_ms") = 2000.0, py::arg("max_ms") = 64000.0,
     py::arg("calm_ms") = 300000.0);
  // The PMC read machine (pmc_rounds.h) on scripted fake GPUs (pmc_fake.h): see
  // tests/test_pmc_rounds.py.  Runs for ticks x tick_us with the GIL released.
  m.def("pmc_agent_lifecycle", [](int gpus, int failing, int starved, int broken, int ticks) {
    gpuexp_pmc::LifecycleOutcome o;
    {
      py::gil_scoped_release nogil;
      o = gpuexp_pmc::run_agent_lifecycle(gpus, failing, starved, broken, ticks);
    }
    py::dict d;
    d["devices"] = o.devices;
    d["matched"] = o.matched;
    d["usable"] = o.usable;
    d["armed"] = o.armed;
    d["queues_created"] = o.queues_created;
    d["queues_live"] = o.queues_live;
    d["signals_created"] = o.signals_created;
    d["signals_live"] = o.signals_live;
    d["buffers_allocated"] = o.buffers_allocated;
    d["buffers_live"] = o.buffers_live;
    d["buffers_left_by_design"] = o.buffers_left_by_design;
    d["double_release"] = o.double_release;
    d["foreign_release"] = o.foreign_release;
    d["rescues_opened"] = o.rescues_opened;
    d["rescues_closed"] = o.rescues_closed;
    d["windows_on_failed_gpu"] = o.windows_on_failed_gpu;
    d["windows"] = o.windows;
    return d;
  }, py::arg("gpus") = 8, py::arg("failing_gpu") = 3, py::arg("starved_gpu") = 5, py::arg("broken_gpu") = 6,
     py::arg("ticks") = 40, "the PMC plugin's multi-agent lifecycle (pmc_agents.h) on stub GPUs");

  m.def("pmc_harness", [](const py::dict& d) {
    using namespace gpuexp_pmc;
    HarnessConfig c;
    auto geti = [&](const char* k, int def) { return d.contains(k) ? d[k].cast<int>() : def; };
    auto getb = [&](const char* k, bool def) { return d.contains(k) ? d[k].cast<bool>() : def; };
    c.gpus = geti("gpus", 8);
    c.ticks = geti("ticks", 60);
    c.tick_us = geti("tick_us", 10000);
    c.work_us = geti("work_us", 300);
    c.sync_us = geti("sync_us", 2000);
    c.inline_rounds = getb("inline", true);
    c.kick_at_end = getb("kick_at_end", false);
    c.reader = getb("reader", true);
    MachineConfig& mc = c.machine;
    const std::string mode = d.contains("mode") ? d["mode"].cast<std::string>() : "cumulative";
    mc.mode = mode == "resets" ? kResets : mode == "stops" ? kStops : kCumulative;
    mc.interval_ms = geti("interval_ms", 1000);
    mc.rescue = getb("rescue", true);
    mc.rescue_rounds = geti("rescue_rounds", 3);
    mc.probation_rounds = geti("probation_rounds", 5);
    mc.first_slice_us = geti("first_slice_us", 60);
    mc.slice_us = geti("slice_us", 100);
    mc.log = getb("log", false);
    const std::string rearm = d.contains("rearm") ? d["rearm"].cast<std::string>() : "backoff";
    mc.rearm.mode = rearm == "off" ? gpuexp_ctr::kRearmOff : rearm == "now" ? gpuexp_ctr::kRearmNow
                                                                            : gpuexp_ctr::kRearmBackoff;
    mc.rearm.base_ns = int64_t(geti("rearm_base_ms", 2000)) * 1000000ll;
    mc.rearm.max_ns = int64_t(geti("rearm_max_ms", 64000)) * 1000000ll;
    if (d.contains("scripts"))
      for (auto item : d["scripts"].cast<py::list>()) {
        py::dict sd = item.cast<py::dict>();
        FakeScript s;
        if (sd.contains("latency_us")) s.latency_us = sd["latency_us"].cast<int64_t>();
        if (sd.contains("stalls")) s.stalls = sd["stalls"].cast<std::vector<std::pair<int64_t, int64_t>>>();
        if (sd.contains("resets")) s.resets = sd["resets"].cast<std::vector<int64_t>>();
        if (sd.contains("stops")) s.stops = sd["stops"].cast<std::vector<std::pair<int64_t, int64_t>>>();
        if (sd.contains("queue_error_at")) s.queue_error_at = sd["queue_error_at"].cast<int64_t>();
        if (sd.contains("rescue_fails")) s.rescue_fails = sd["rescue_fails"].cast<bool>();
        if (sd.contains("rate")) s.rate = sd["rate"].cast<double>();
        if (sd.contains("read_mode")) s.read_mode = sd["read_mode"].cast<int>();
        c.scripts.push_back(s);
      }
    const double tol = d.contains("rate_tolerance") ? d["rate_tolerance"].cast<double>() : 0.1;
    HarnessOutcome o;
    {
      py::gil_scoped_release nogil;
      o = run_pmc_harness(c, tol);
    }
    py::dict r;
    r["ticks"] = o.ticks;
    r["late_syncs"] = o.late_syncs;
    r["max_sync_us"] = o.max_sync_us;
    r["max_kick_us"] = o.max_kick_us;
    r["reader_calls"] = o.reader_calls;
    r["armed_all"] = o.armed_all;
    py::list gl;
    for (auto& g : o.gpus) {
      py::dict x;
      x["stalls"] = g.health.stalls;
      x["resets"] = g.health.resets;
      x["rearms"] = g.health.rearms;
      x["rescues"] = g.health.rescues;
      x["releases"] = g.health.releases;
      x["rescue_active"] = g.health.rescue_active;
      x["waiting_rearm"] = g.health.waiting_rearm;
      x["conflicts"] = g.health.conflicts;
      x["broken"] = g.health.broken;
      x["windows"] = g.windows;
      x["fresh_ticks"] = g.fresh_ticks;
      x["bad_windows"] = g.bad_windows;
      x["worst_rate_err"] = g.worst_rate_err;
      x["packets"] = g.packets;
      x["reads_completed"] = g.reads_completed;
      x["uncollected"] = g.uncollected;
      x["double_collected"] = g.double_collected;
      x["arms"] = g.arms;
      x["max_lateness_us"] = g.max_lateness_us;
      x["rescue_opened"] = g.rescue_opened;
      x["rescue_closed"] = g.rescue_closed;
      x["misuse"] = g.misuse;
      x["rescue_open_at_end"] = g.rescue_open_at_end;
      gl.append(x);
    }
    r["gpus"] = gl;
    return r;
  });
  m.def("counter_names", []() {
    std::vector<std::string> v;
    for (int k = 0; k < gpuexp_ctr::kNumCtr; ++k) v.push_back(gpuexp_ctr::name(k));
    return v;
  });
  m.def("uuid_from_unique_id", &SysfsBackend::uuid_from_unique_id);
  m.def("parse_ras_err_count", [](const std::string& body) {
    RasTotals t;
    bool ok = parse_ras_err_count(body, &t);
    py::dict d;
    d["ok"] = ok;
    d["ce"] = t.ecc_ce;
    d["ue"] = t.ecc_ue;
    d["de"] = t.ecc_de;
    return d;
  });
  m.def("parse_aer_total", &parse_aer_total);
  m.def("read_backend", [](const std::string& backend, const std::string& host_root, int ndev) {
    // One-shot enumerate + sample (diagnostics / tests).
    std::unique_ptr<Backend> b;
    if (backend == "sysfs") b = std::make_unique<SysfsBackend>(host_root);
    else if (backend == "amdsmi") b = make_amdsmi_backend(host_root, true, false);
    else b = std::make_unique<MockBackend>(ndev);
    std::vector<DeviceInfo> devs;
    std::string err;
    py::list out;
    bool ok;
    {
      py::gil_scoped_release rel;
      ok = b->init(&devs, &err);
    }
    if (!ok) throw std::runtime_error(err);
    for (auto& d : devs) {
      DeviceSample s;
      s.host_ns = mono_ns();
      b->sample(d, &s);
      py::dict e = device_dict(d);
      e["sample"] = sample_dict(s);
      e["source"] = b->describe(d);
      std::vector<ProcSample> procs;
      py::list pl;
      if (b->processes(d, &procs))
        for (auto& p : procs) {
          py::dict pd;
          pd["pid"] = p.pid;
          pd["vram_bytes"] = p.vram_bytes;
          pd["cu_occupancy"] = p.cu_occupancy;
          pd["name"] = p.name;
          pl.append(pd);
        }
      e["processes"] = pl;
      out.append(e);
    }
    b->shutdown();
    return out;
  }, py::arg("backend"), py::arg("host_root") = "", py::arg("ndev") = 1);
  m.def("scan_kfd", [](const std::string& host_root, std::vector<uint32_t> gpu_ids, int self_pid) {
    std::vector<DeviceInfo> devs;
    for (size_t i = 0; i < gpu_ids.size(); ++i) {
      DeviceInfo d;
      d.index = int(i);
      d.kfd_gpu_id = gpu_ids[i];
      devs.push_back(d);
    }
    KfdProcReader r(host_root, self_pid, true);
    std::vector<std::vector<ProcSample>> per;
    r.scan(devs, &per);
    py::list out;
    for (auto& l : per) {
      py::list dl;
      for (auto& p : l) {
        py::dict pd;
        pd["pid"] = p.pid;
        pd["vram_bytes"] = p.vram_bytes;
        pd["cu_occupancy"] = p.cu_occupancy;
        pd["sdma_us"] = p.sdma_us;
        pd["name"] = p.name;
        dl.append(pd);
      }
      out.append(dl);
    }
    return out;
  }, py::arg("host_root"), py::arg("gpu_ids"), py::arg("self_pid") = -1);

  m.def("scrape_loop", [](const std::string& host, int port, const std::string& path, double hz, int count,
                          bool gzip, bool keepalive, int timeout_ms, bool keep_last_body) {
    ScrapeResult r;
    {
      py::gil_scoped_release rel;
      r = scrape_loop(host, port, path, hz, count, gzip, keepalive, timeout_ms, keep_last_body);
    }
    py::dict d;
    d["latency_ns"] = r.latency_ns;
    d["bytes"] = r.bytes;
    d["errors"] = r.errors;
    d["non200"] = r.non200;
    d["wall_s"] = r.wall_s;
    d["last_body"] = py::bytes(r.last_body);
    return d;
  }, py::arg("host"), py::arg("port"), py::arg("path") = "/metrics", py::arg("hz") = 10.0,
     py::arg("count") = 100, py::arg("gzip") = false, py::arg("keepalive") = true,
     py::arg("timeout_ms") = 5000, py::arg("keep_last_body") = false);

  m.def("scrape_period_ns", [](std::vector<uint64_t> newest_first) {
    return learnt_scrape_period_ns(newest_first.data(), int(std::min<size_t>(newest_first.size(), 4)));
  }, py::arg("intervals_newest_first"), "The scrape period the HTTP pre-wake learns from request intervals (ns)");

  m.def("spin_windows", [](std::vector<uint64_t> arrivals, uint64_t max_ns, uint64_t margin) {
    // replays arrivals through the spin pre-wake's predictor: for each arrival after the
    // first, the window it would have been polled in (from, until, predictor) -- 0s = none
    ArrivalPredictor p;
    py::list out;
    for (size_t i = 0; i < arrivals.size(); ++i) {
      if (i) {
        uint64_t f = 0, u = 0;
        const int which = p.window(max_ns, margin, &f, &u);
        out.append(py::make_tuple(f, u, which));
      }
      p.observe(arrivals[i], true);
    }
    return out;
  }, py::arg("arrivals_ns"), py::arg("max_ns") = 300000, py::arg("margin_ns") = 15000,
     "Spin pre-wake windows (ArrivalPredictor, http.h) for a sequence of request arrivals");

  py::class_<ScrapeClient>(m, "ScrapeClient")
      .def(py::init<std::string, int, std::string, bool, int, std::string, bool>(), py::arg("host"),
           py::arg("port"), py::arg("path") = "/metrics", py::arg("gzip") = false, py::arg("timeout_ms") = 5000,
           py::arg("accept") = "", py::arg("timing") = false)
      .def("scrape", [](ScrapeClient& c) {
        py::gil_scoped_release rel;
        return c.scrape();
      })
      .def_property_readonly("last_status", &ScrapeClient::last_status)
      .def_property_readonly("last_bytes", &ScrapeClient::last_bytes)
      .def_property_readonly("errors", &ScrapeClient::errors)
      .def("last_body", [](ScrapeClient& c) { return py::bytes(c.last_body()); })
      .def("last_server_rx", &ScrapeClient::last_server_rx,
           "CLOCK_MONOTONIC ns when the server's kernel queued the last request (0 = unknown)")
      .def("last_prewoken", &ScrapeClient::last_prewoken,
           "1 if the server's worker was pre-woken for the last request, 0 if not, -1 unknown")
      .def("last_timing", &ScrapeClient::last_timing,
           "CLOCK_MONOTONIC ns [client send, server parsed, server writing, client done] of the last scrape");

  // --- SeriesTable (unit tests of the exposition layer) ---
  py::enum_<MetricType>(m, "MetricType")
      .value("gauge", MetricType::kGauge)
      .value("counter", MetricType::kCounter)
      .value("histogram", MetricType::kHistogram);
  py::class_<SeriesTable>(m, "SeriesTable")
      .def(py::init<>())
      .def("add_family", [](SeriesTable& t, const std::string& name, const std::string& help, MetricType type,
                            std::vector<std::string> labels) {
        return t.add_family(FamilyDef{name, help, type, std::move(labels)});
      })
      .def("put", &SeriesTable::put)
      .def("observe", [](SeriesTable& t, int fid, std::vector<std::string> labels, double v, uint64_t gen,
                         std::vector<double> bounds) {
        t.observe(t.upsert(fid, labels), v, gen, bounds);
      })
      .def("render", [](SeriesTable& t, uint64_t gen, uint64_t gc_after) {
        std::string out;
        t.render(&out, gen, gc_after);
        return out;
      }, py::arg("gen"), py::arg("gc_after") = 1)
      .def("render_compiled", [](SeriesTable& t, uint64_t gen, uint64_t gc_after, bool gzip) {
        std::string out, gz;
        t.render_compiled(&out, gzip ? &gz : nullptr, gen, gc_after);
        return py::make_tuple(out, py::bytes(gz));
      }, py::arg("gen"), py::arg("gc_after") = 1, py::arg("gzip") = true,
         "(text, gzip bytes) of the fixed-layout renderer")
      .def("render_compiled_slot", [](SeriesTable& t, uint64_t gen, int slot, uint64_t gc_after) {
        // the engine's snapshot slots: buffers kept between calls, each with the generation it holds
        static thread_local std::map<std::pair<const SeriesTable*, int>, std::pair<std::string, uint64_t>> slots;
        auto& sl = slots[{&t, slot}];
        std::string gz;
        t.render_compiled(&sl.first, &gz, gen, gc_after, sl.second);
        sl.second = gen;
        return py::make_tuple(sl.first, py::bytes(gz), t.last_copied());
      }, py::arg("gen"), py::arg("slot"), py::arg("gc_after") = 1,
         "render_compiled into a kept buffer (slot): (text, gzip, bytes copied into the buffer)")
      .def("last_relayouts", &SeriesTable::last_relayouts)
      .def("last_skipped", &SeriesTable::last_skipped)
      .def("provisional_parses", &SeriesTable::provisional_parses)
      .def("code_builds", &SeriesTable::code_builds)
      .def("set_histogram", [](SeriesTable& t, int fid, std::vector<std::string> labels, std::vector<double> bounds,
                               std::vector<uint64_t> counts, double sum, uint64_t count, uint64_t gen) {
        t.set_histogram(t.upsert(fid, labels), bounds, counts, sum, count, gen);
      })
      .def("live_series", &SeriesTable::live_series);

  // --- Engine ---
  py::class_<HttpConfig>(m, "HttpConfig")
      .def(py::init<>())
      .def_readwrite("host", &HttpConfig::host)
      .def_readwrite("port", &HttpConfig::port)
      .def_readwrite("metrics_path", &HttpConfig::metrics_path)
      .def_readwrite("threads", &HttpConfig::threads)
      .def_readwrite("max_conns", &HttpConfig::max_conns)
      .def_readwrite("idle_timeout_ms", &HttpConfig::idle_timeout_ms)
      .def_readwrite("enable_gzip", &HttpConfig::enable_gzip)
      .def_readwrite("gzip_unsteady_hold_ns", &HttpConfig::gzip_unsteady_hold_ns)
      .def_readwrite("socket_sndbuf", &HttpConfig::socket_sndbuf)
      .def_readwrite("stale_after_ns", &HttpConfig::stale_after_ns)
      // legacy boolean: True = the timer-slice mode, False = off
      .def_property("prewake", [](const HttpConfig& h) { return h.prewake_mode != kPrewakeOff; },
                    [](HttpConfig& h, bool on) { h.prewake_mode = on ? kPrewakeSlices : kPrewakeOff; })
      .def_property("prewake_mode", [](const HttpConfig& h) { return std::string(prewake_mode_name(h.prewake_mode)); },
                    [](HttpConfig& h, const std::string& m) {
                      const int v = parse_prewake_mode(m);
                      if (v < 0) throw py::value_error("prewake_mode must be off|slices|spin, got " + m);
                      h.prewake_mode = v;
                    })
      .def_readwrite("prewake_spin_max_ns", &HttpConfig::prewake_spin_max_ns)
      .def_readwrite("prewake_spin_margin_ns", &HttpConfig::prewake_spin_margin_ns)
      .def_readwrite("follow_rx_cpu", &HttpConfig::follow_rx_cpu)
      .def_readwrite("prewake_lead_ns", &HttpConfig::prewake_lead_ns)
      .def_readwrite("prewake_step_ns", &HttpConfig::prewake_step_ns)
      .def_readwrite("prewake_window_ns", &HttpConfig::prewake_window_ns);

  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("backend", &EngineConfig::backend)
      .def_readwrite("device_threads", &EngineConfig::device_threads)
      .def_readwrite("mock_devices", &EngineConfig::mock_devices)
      .def_readwrite("mock_xgmi_file", &EngineConfig::mock_xgmi_file)
      .def_readwrite("host_root", &EngineConfig::host_root)
      .def_readwrite("interval_s", &EngineConfig::interval_s)
      .def_readwrite("serve_http", &EngineConfig::serve_http)
      .def_readwrite("http", &EngineConfig::http)
      .def_readwrite("series_profile", &EngineConfig::series_profile)
      .def_readwrite("ras_interval_s", &EngineConfig::ras_interval_s)
      .def_readwrite("metrics_coalesce", &EngineConfig::metrics_coalesce)
      .def_readwrite("legacy_families", &EngineConfig::legacy_families)
      .def_readwrite("pod_attribution", &EngineConfig::pod_attribution)
      .def_readwrite("infer_device_owner", &EngineConfig::infer_device_owner)
      .def_readwrite("process_source", &EngineConfig::process_source)
      .def_readwrite("kfd_cu_occupancy", &EngineConfig::kfd_cu_occupancy)
      .def_readwrite("kfd_sdma", &EngineConfig::kfd_sdma)
      .def_readwrite("kfd_detail_interval_s", &EngineConfig::kfd_detail_interval_s)
      .def_readwrite("exclude_self", &EngineConfig::exclude_self)
      .def_readwrite("enable_sentinel", &EngineConfig::enable_sentinel)
      .def_readwrite("sentinel_impl", &EngineConfig::sentinel_impl)
      .def_readwrite("sentinel_ring", &EngineConfig::sentinel_ring)
      .def_readwrite("sentinel_spin", &EngineConfig::sentinel_spin)
      .def_readwrite("enable_counters", &EngineConfig::enable_counters)
      .def_readwrite("counters_plugin", &EngineConfig::counters_plugin)
      .def_readwrite("counters_mode", &EngineConfig::counters_mode)
      .def_readwrite("counters_sync_us", &EngineConfig::counters_sync_us)
      .def_readwrite("counters_kick", &EngineConfig::counters_kick)
      .def_readwrite("counters_inline", &EngineConfig::counters_inline)
      .def_readwrite("counters_window_ms", &EngineConfig::counters_window_ms)
      .def_readwrite("counters_interval_ms", &EngineConfig::counters_interval_ms)
      .def_readwrite("enable_rccl", &EngineConfig::enable_rccl)
      .def_readwrite("rccl_dir", &EngineConfig::rccl_dir)
      .def_readwrite("rccl_verify", &EngineConfig::rccl_verify)
      .def_readwrite("rccl_scan_interval_s", &EngineConfig::rccl_scan_interval_s)
      .def_readwrite("enable_kfd_events", &EngineConfig::enable_kfd_events)
      .def_readwrite("firmware_info", &EngineConfig::firmware_info)
      .def_readwrite("state_file", &EngineConfig::state_file)
      .def_readwrite("state_interval_s", &EngineConfig::state_interval_s)
      .def_readwrite("kfd_path", &EngineConfig::kfd_path)
      .def_readwrite("metrics_min_interval_s", &EngineConfig::metrics_min_interval_s)
      .def_readwrite("metrics_cpu_budget", &EngineConfig::metrics_cpu_budget)
      .def_readwrite("pod_totals_ttl_s", &EngineConfig::pod_totals_ttl_s)
      .def_readwrite("kfd_rescan_interval_s", &EngineConfig::kfd_rescan_interval_s)
      .def_readwrite("metrics_max_interval_s", &EngineConfig::metrics_max_interval_s)
      .def_readwrite("fake_metrics_cost_us", &EngineConfig::fake_metrics_cost_us)
      .def_readwrite("fake_pmc_cost_us", &EngineConfig::fake_pmc_cost_us)
      .def_readwrite("fake_pmc_stalls_us", &EngineConfig::fake_pmc_stalls_us)
      .def_readwrite("fake_sentinel_cost_us", &EngineConfig::fake_sentinel_cost_us)
      .def_readwrite("sampler_thread", &EngineConfig::sampler_thread)
      .def_readwrite("render_when_due", &EngineConfig::render_when_due)
      .def_readwrite("render_every_ticks", &EngineConfig::render_every_ticks)
      .def_readwrite("process_min_interval_s", &EngineConfig::process_min_interval_s)
      .def_readwrite("sentinel_min_interval_s", &EngineConfig::sentinel_min_interval_s)
      .def_readwrite("counters_min_interval_s", &EngineConfig::counters_min_interval_s)
      .def_readwrite("counters_cpu_budget", &EngineConfig::counters_cpu_budget)
      .def_readwrite("queue_devices", &EngineConfig::queue_devices)
      .def_readwrite("queue_devices_bdf", &EngineConfig::queue_devices_bdf)
      .def_readwrite("force_amdsmi_metrics", &EngineConfig::force_amdsmi_metrics)
      .def_readwrite("gzip_level", &EngineConfig::gzip_level)
      .def_readwrite("exposition", &EngineConfig::exposition)
      .def_readwrite("gc_after", &EngineConfig::gc_after)
      .def_readwrite("device_filter", &EngineConfig::device_filter)
      .def_readwrite("device_filter_bdf", &EngineConfig::device_filter_bdf)
      .def_readwrite("trace_path", &EngineConfig::trace_path)
      .def_readwrite("trace_max_events", &EngineConfig::trace_max_events)
      .def_readwrite("version", &EngineConfig::version);

  py::class_<Engine>(m, "Engine")
      .def(py::init<const EngineConfig&>())
      .def("start", [](Engine& e) {
        std::string err;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = e.start(&err);
        }
        if (!ok) throw std::runtime_error("engine start failed: " + err);
      })
      .def("stop", [](Engine& e) {
        py::gil_scoped_release rel;
        e.stop();
      })
      .def("tick", [](Engine& e, py::object now_ns) {
        uint64_t t = now_ns.is_none() ? mono_ns() : now_ns.cast<uint64_t>();
        py::gil_scoped_release rel;
        e.tick_now(t);
      }, py::arg("now_ns") = py::none())
      .def("snapshot_text", [](Engine& e) {
        std::string s;
        {
          py::gil_scoped_release rel;
          s = e.snapshot_text();
        }
        return s;
      })
      .def_property_readonly("http_port", &Engine::http_port)
      .def("devices", [](Engine& e) {
        py::list l;
        for (auto& d : e.devices()) l.append(device_dict(d));
        return l;
      })
      .def("stats", [](Engine& e) {
        EngineStats s = e.stats();
        py::dict d;
        d["ticks"] = s.ticks;
        d["overruns"] = s.overruns;
        d["publish_skipped"] = s.publish_skipped;
        d["last_tick_ns"] = s.last_tick_ns;
        d["max_tick_ns"] = s.max_tick_ns;
        d["tick_ns_total"] = s.tick_ns_total;
        d["max_tick_cpu_ns"] = s.max_tick_cpu_ns;
        d["tick_cpu_ns_total"] = s.tick_cpu_ns_total;
        d["fake_cpu_burnt_ns"] = fake_cpu_burnt_ns().load();  // (process-wide: the fake sources' stand-ins)
        d["fresh_reads"] = s.fresh_reads;
        d["last_tick_fresh"] = s.last_tick_fresh;
        d["sentinel_runs"] = s.sentinel_runs;
        d["kfd_lists"] = s.kfd_lists;
        d["leveled_ticks"] = s.leveled_ticks;
        d["renders_skipped"] = s.renders_skipped;
        d["counter_rounds"] = s.counter_rounds;
        d["counters_round_cpu_ns"] = s.counters_round_cpu_ns;
        d["counters_round_interval_s"] = s.counters_round_interval_s;
        d["render_bytes"] = s.render_bytes;
        d["series"] = s.series;
        d["device_errors"] = s.device_errors;
        d["sampler_cpu_ns"] = s.sampler_cpu_ns;
        d["gzip_eager"] = s.gzip_eager;
        d["relayouts"] = s.relayouts;
        d["code_builds"] = s.code_builds;
        d["families_skipped"] = s.families_skipped;
        d["families_rendered"] = s.families_rendered;
        py::dict st;
        for (int k = 0; k < Engine::kStages; ++k) st[Engine::stage_name(k)] = s.stage_ns[k];
        d["stage_ns"] = st;
        py::dict sc;
        for (int k = 0; k < Engine::kStages; ++k) sc[Engine::stage_name(k)] = s.stage_cpu_ns[k];
        d["stage_cpu_ns"] = sc;
        if (const HttpStats* hs = e.http_stats()) {
          d["http_requests"] = hs->requests.load();
          d["http_metrics_requests"] = hs->metrics_requests.load();
          d["http_gzip_responses"] = hs->gzip_responses.load();
          d["http_gzip_on_demand"] = hs->gzip_on_demand.load();
          d["http_rx_cpu_moves"] = hs->rx_cpu_moves.load();
          d["http_bytes"] = hs->bytes_sent.load();
          d["http_errors"] = hs->errors.load();
          d["http_open_conns"] = hs->open_conns.load();
          d["http_writev_calls"] = hs->writev_calls.load();
          d["http_prewake_timer_wakeups"] = hs->prewake_timer_wakeups.load();
          d["http_prewake_hits"] = hs->prewake_hits.load();
          d["http_prewake_hits_narrow"] = hs->prewake_hits_narrow.load();
          d["http_prewake_spins"] = hs->prewake_spins.load();
          d["http_prewake_spin_hits"] = hs->prewake_spin_hits.load();
          d["http_prewake_spin_timeouts"] = hs->prewake_spin_timeouts.load();
          d["http_prewake_spin_ns"] = hs->prewake_spin_ns.load();
          d["http_writev_ns"] = hs->writev_ns.load();
          d["http_partial_writes"] = hs->partial_writes.load();
          d["http_scrape_ns"] = hs->lat_sum_ns.load();
          d["http_scrapes"] = hs->lat_count.load();
        }
        return d;
      })
      .def("set_prewake_mode", [](Engine& e, const std::string& m) {
        const int v = parse_prewake_mode(m);
        if (v < 0) throw py::value_error("prewake mode must be off|slices|spin, got " + m);
        return e.set_prewake_mode(v);
      }, py::arg("mode"), "switch the HTTP workers' scrape pre-wake at run time (off|slices|spin)")
      .def_property_readonly("prewake_mode", [](const Engine& e) { return std::string(prewake_mode_name(e.prewake_mode())); })
      .def("reset_tick_max", &Engine::reset_tick_max, "restart stats()['max_tick_ns'] and ['max_tick_cpu_ns'] (a measurement window)")
      .def("source_status", &Engine::source_status)
      .def("set_pods", [](Engine& e, py::list pods, bool complete) {
        std::vector<PodMeta> v;
        for (auto item : pods) {
          py::dict d = item.cast<py::dict>();
          PodMeta p;
          p.uid = d["uid"].cast<std::string>();
          p.ns = d["namespace"].cast<std::string>();
          p.name = d["name"].cast<std::string>();
          if (d.contains("containers"))
            for (auto kv : d["containers"].cast<py::dict>())
              p.containers.emplace_back(kv.first.cast<std::string>(), kv.second.cast<std::string>());
          v.push_back(std::move(p));
        }
        e.set_pods(std::move(v), complete);
      }, py::arg("pods"), py::arg("complete") = true,
         "complete=False: a source failed this refresh; the list is applied for names but never used to "
         "drop per-pod totals")
      .def("set_device_owners", [](Engine& e, py::dict owners) {
        std::vector<std::pair<std::string, DeviceOwner>> v;
        for (auto kv : owners) {
          py::dict o = kv.second.cast<py::dict>();
          DeviceOwner d;
          d.ns = o.contains("namespace") ? o["namespace"].cast<std::string>() : "";
          d.pod = o.contains("pod") ? o["pod"].cast<std::string>() : "";
          d.container = o.contains("container") ? o["container"].cast<std::string>() : "";
          v.emplace_back(kv.first.cast<std::string>(), d);
        }
        e.set_device_owners(std::move(v));
      })
      .def("set_pid_cgroup", &Engine::set_pid_cgroup)
      .def("inject_kfd_events", [](Engine& e, int dev, py::bytes b) { e.inject_kfd_events(dev, std::string(b)); },
           "Test hook: bytes as if read from GPU `dev`'s KFD SMI event fd (counted at the next tick)")
      .def("clear_pid_cgroups", &Engine::clear_pid_cgroups)
      .def("mock_set_value", [](Engine& e, int dev, const std::string& field, double v) {
        if (!e.mock()) throw std::runtime_error("not a mock backend");
        e.mock()->set_value(dev, field, v);
      })
      .def("mock_set_processes", [](Engine& e, int dev, py::list procs) {
        if (!e.mock()) throw std::runtime_error("not a mock backend");
        std::vector<ProcSample> v;
        for (auto item : procs) v.push_back(proc_from_dict(item.cast<py::dict>()));
        e.mock()->set_processes(dev, v);
      })
      .def("mock_clear_processes", [](Engine& e) {
        if (!e.mock()) throw std::runtime_error("not a mock backend");
        e.mock()->clear_processes();
      })
      .def("mock_set_fault", [](Engine& e, int dev, const std::string& fault) {
        if (!e.mock()) throw std::runtime_error("not a mock backend");
        e.mock()->set_fault(dev, fault);
      });

  m.def("default_rocprof_plugin", &default_rocprof_plugin);
}
