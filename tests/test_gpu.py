"""Real-MI355X tier (BASELINE configs 2-5 on one GPU): amdsmi backend + raw gpu_metrics
fast path, HIP sentinel, MFMA GEMM numerics, KFD process discovery under a live workload.
Every test here runs the native (HIP / amdsmi) path — nothing falls back to Python."""
import os
import subprocess
import sys
import time

import pytest

from kubernetes_gpu_exporter_amd.ops.gemm import kernels
from kubernetes_gpu_exporter_amd.utils import promtext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def amdsmi_engine(native, **kw):
    c = native.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0
    c.serve_http = False
    c.device_filter = [0]
    for k, v in kw.items():
        setattr(c, k, v)
    e = native.Engine(c)
    e.start()
    return e


def test_amdsmi_backend_and_fast_path(native):
    devs = native.read_backend("amdsmi")
    assert len(devs) >= 1
    d = devs[0]
    print("device:", {k: d[k] for k in ("bdf", "uuid", "name", "kfd_gpu_id", "render_minor", "vram_total")})
    print("source:", d["source"])
    s = d["sample"]
    assert s["ok"]
    assert d["vram_total"] > 250 * (1 << 30)  # 288 GB HBM3E
    assert 0 <= s["gfx_activity"] <= 100
    assert 10 < s["temp_hotspot"] < 120
    assert 50 < s["power_w"] < 2000
    assert s["vram_max_bw_gbs"] > 1000
    assert "validated" in d["source"], d["source"]
    # partition identity from amdsmi (SPX/NPS1 on the gpurun boxes; CPX splits a socket)
    print("partition:", {k: d[k] for k in ("partition_id", "compute_partition", "memory_partition", "num_xcc")})
    assert d["compute_partition"] in ("SPX", "DPX", "QPX", "CPX"), d
    assert d["memory_partition"].startswith("NPS"), d
    assert d["num_xcc"] == {"SPX": 8, "DPX": 4, "QPX": 2, "CPX": 1}[d["compute_partition"]], d


# gpu_metrics v1.8 fields by how a correct decode relates to two amdsmi reads around it
_ACC = ["energy_accumulator", "system_clock_counter", "accumulation_counter", "prochot_residency_acc",
        "ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc", "hbm_thm_residency_acc",
        "gfx_activity_acc", "mem_activity_acc", "pcie_bandwidth_acc", "pcie_l0_to_recov_count_acc",
        "pcie_replay_count_acc", "pcie_replay_rover_count_acc", "pcie_nak_sent_count_acc",
        "pcie_nak_rcvd_count_acc", "firmware_timestamp", "xgmi_read_data_acc", "xgmi_write_data_acc",
        "xcp_stats.gfx_busy_acc"]
_STATIC = ["vram_max_bandwidth", "pcie_link_width", "pcie_link_speed", "xgmi_link_width", "xgmi_link_speed",
           "num_partition", "xgmi_link_status", "current_uclk"]
_NEAR = {"temperature_hotspot": 3, "temperature_mem": 3, "temperature_vrsoc": 3, "current_socket_power": 100,
         "average_gfx_activity": 25, "average_umc_activity": 25, "current_gfxclks": 400, "current_socclks": 400,
         "pcie_bandwidth_inst": 64}


def _flat(v):
    if isinstance(v, list):
        return [x for e in v for x in _flat(e)]
    return [v]


def test_raw_gpu_metrics_matches_amdsmi_python(native):
    """Field-by-field parity of the raw v1.8 decoder with the amdsmi Python binding (an
    independent ctypes layout): every exported accumulator lies between two amdsmi reads
    taken around the raw read, static fields agree exactly, sensors within their jitter,
    and "N/A" in amdsmi is the all-ones sentinel in the raw blob.  Then the converted
    DeviceSample (what the engine exports) is checked against the raw fields."""
    amdsmi = pytest.importorskip("amdsmi")
    import time
    os.environ.setdefault("AMDSMI_GPU_METRICS_CACHE_MS", "0")  # amdsmi caches tables otherwise

    def na_ok(name, r, a):  # amdsmi's "N/A" = the blob field's all-ones sentinel, at its own width
        return a == "N/A" and r in (0xFFFF, 0xFFFFFFFF, (1 << 64) - 1)

    def compare(m1, raw, m2):
        checked, problems = [], []
        for name in _ACC + _STATIC + list(_NEAR):
            a1, r, a2 = _flat(m1[name]), _flat(raw[name]), _flat(m2[name])
            if name == "xcp_stats.gfx_busy_acc":  # amdsmi lists 8 partitions x 8 XCDs, as the blob
                a1, a2 = a1[:len(r)], a2[:len(r)]
            assert len(a1) == len(r) == len(a2), (name, len(a1), len(r))
            for lo, v, hi in zip(a1, r, a2):
                if "N/A" in (lo, hi):
                    ok = na_ok(name, v, lo if lo == "N/A" else hi)
                elif name in _ACC:
                    ok = lo <= v <= hi
                elif name in _STATIC:
                    ok = lo == v == hi
                else:
                    ok = min(lo, hi) - _NEAR[name] <= v <= max(lo, hi) + _NEAR[name]
                if not ok:
                    problems.append((name, lo, v, hi))
            checked.append(name)
        return checked, problems

    amdsmi.amdsmi_init()
    try:
        h = amdsmi.amdsmi_get_processor_handles()[0]
        info = native.read_backend("amdsmi")[0]
        path = f"/sys/class/drm/renderD{info['render_minor']}/device/gpu_metrics"
        for attempt in range(3):  # a bracket can straddle a PMFW refresh oddly: retry, 30 ms apart
            m1 = amdsmi.amdsmi_get_gpu_metrics_info(h)
            time.sleep(0.01)
            with open(path, "rb") as fh:
                blob = fh.read()
            time.sleep(0.01)
            m2 = amdsmi.amdsmi_get_gpu_metrics_info(h)
            raw = native.decode_gpu_metrics_raw(blob)
            assert raw is not None
            checked, problems = compare(m1, raw, m2)
            print(f"attempt {attempt}: {len(checked)} gpu_metrics fields checked against amdsmi; mismatches: {problems}")
            if not problems:
                break
            time.sleep(0.03)
        e = amdsmi.amdsmi_get_energy_count(h)
    finally:
        amdsmi.amdsmi_shut_down()
    assert not problems, problems
    assert len(checked) >= 25

    # the converted sample the engine exports
    s = native.decode_gpu_metrics(blob)
    assert s["energy_acc"] == raw["energy_accumulator"] and s["energy_valid"]
    assert s["accumulation_counter"] == raw["accumulation_counter"]
    for k, r in (("res_ppt", "ppt_residency_acc"), ("res_prochot", "prochot_residency_acc"),
                 ("res_socket_thm", "socket_thm_residency_acc"), ("res_vr_thm", "vr_thm_residency_acc"),
                 ("res_hbm_thm", "hbm_thm_residency_acc"), ("pcie_bw_acc", "pcie_bandwidth_acc")):
        assert s[k] == raw[r], k
    assert s["pcie_speed_gts"] == raw["pcie_link_speed"] / 10.0 and s["pcie_width"] == raw["pcie_link_width"]
    assert s["xgmi_width"] == raw["xgmi_link_width"] and s["xgmi_speed"] == raw["xgmi_link_speed"]
    assert s["fw_ts_10ns"] == raw["firmware_timestamp"]
    assert s["gfx_busy_acc"] == raw["xcp_stats.gfx_busy_acc"][0]
    assert s["xgmi_read_kb"] == [0 if v == (1 << 64) - 1 else v for v in raw["xgmi_read_data_acc"]]
    assert s["clk_mem"] == raw["current_uclk"] and s["vram_max_bw_gbs"] == raw["vram_max_bandwidth"]
    assert [c for c in s["clk_gfx_xcc"] if c == c] == [c for c in raw["current_gfxclks"] if c not in (0, 0xFFFF)]
    for k, r in (("pcie_nak_sent", "pcie_nak_sent_count_acc"), ("pcie_nak_rcvd", "pcie_nak_rcvd_count_acc"),
                 ("pcie_l0_recov", "pcie_l0_to_recov_count_acc"), ("pcie_replay", "pcie_replay_count_acc")):
        assert s[k] == raw[r] or (s[k] != s[k] and raw[r] in ((1 << 32) - 1, (1 << 64) - 1)), k
    # energy: the exporter's joules = accumulator x 15.259 uJ, as amdsmi_get_energy_count says
    print("amdsmi energy count:", e)
    res = e.get("counter_resolution")
    if isinstance(res, (int, float)) and res > 0:
        assert abs(res - 15.259) < 0.1, res


def test_exporter_tick_on_gpu(native):
    e = amdsmi_engine(native, enable_sentinel=True)
    try:
        for _ in range(5):
            e.tick()
            time.sleep(0.05)
        text = e.snapshot_text()
        fams = promtext.parse(text)
        assert promtext.value(fams, "amd_gpu_up", gpu=0) == 1
        vram = promtext.value(fams, "amd_gpu_vram_total_bytes", gpu=0)
        assert vram > 250e9
        print(e.source_status())
        print(e.stats())
        sclk = promtext.value(fams, "amd_gpu_sentinel_sclk_hz", gpu=0)
        assert 50e6 < sclk < 3.0e9, sclk
        runs = promtext.value(fams, "amd_gpu_sentinel_runs_total", gpu=0)
        assert runs >= 2
        try:
            lat = promtext.value(fams, "amd_gpu_sentinel_dispatch_latency_seconds", gpu=0)
            print("sentinel dispatch latency", lat)
            assert 0 <= lat < 0.5
        except KeyError:
            pytest.fail("sentinel latency not exported (tick domain mismatch?)")
        xcc = promtext.value(fams, "amd_gpu_sentinel_xcc_id", gpu=0)
        assert 0 <= xcc < 8
    finally:
        e.stop()


def test_counters_at_100hz_read_kicked_at_the_previous_tick_end(native):
    """A 100 Hz engine (counters_kick auto -> "end"): each tick's PMC read goes out at the end
    of the previous tick, so it has completed by the counters stage -- the stage stays short,
    no tick misses its window, and the counter families are exported
    (profiles/r04/kick_end_100hz.txt)."""
    from kubernetes_gpu_exporter_amd._native import rocprof_plugin_path
    e = amdsmi_engine(native, interval_s=0.01, enable_counters=True, enable_sentinel=True,
                      counters_plugin=rocprof_plugin_path("aqlpmc"), series_profile="full")
    try:
        if "counters=unavailable" in e.source_status():
            pytest.skip("device counting unavailable on this box: " + e.source_status())
        time.sleep(0.5)
        s0 = e.stats()
        time.sleep(2.0)
        s1 = e.stats()
        fams = promtext.parse(e.snapshot_text())
    finally:
        e.stop()
    ticks = s1["ticks"] - s0["ticks"]
    counters_us = (s1["stage_cpu_ns"]["counters"] - s0["stage_cpu_ns"]["counters"]) / max(1, ticks) / 1e3
    late = promtext.value(fams, "gpuexp_counters_late_ticks_total")
    print(f"{ticks} ticks, counters stage {counters_us:.1f} us CPU per tick, late {late}")
    assert ticks > 150
    assert promtext.value(fams, "amd_gpu_gui_active_percent", gpu=0) >= 0
    assert promtext.value(fams, "amd_gpu_mfma_busy_percent", gpu=0) >= 0
    assert late <= 0.05 * s1["ticks"], late
    assert counters_us < 100, counters_us


def test_devices_stage_split_on_mi355x(native):
    """The devices stage split on real hardware: a fresh gpu_metrics read is an SMU round trip
    the kernel busy-waits on, so its thread CPU is tens to hundreds of microseconds (idle:
    ~206 us, profiles/r03/read_costs.txt), it is the bulk of the stage, and the auto fetch
    policy at 1 GPU caps nothing at 10 Hz (one GPU's fetches fit the 1.5 % budget)."""
    e = amdsmi_engine(native, series_profile="full", interval_s=0.1)
    try:
        time.sleep(2.0)
        fams = promtext.parse(e.snapshot_text())
        st = e.stats()
    finally:
        e.stop()
    parts = {lab["part"]: v for _, lab, v in promtext.samples(fams, "gpuexp_device_read_seconds_total")}
    assert set(parts) == {"counters_kick", "control", "gpu_metrics", "vram", "ras", "gtt"}, parts
    fresh = promtext.value(fams, "gpuexp_gpu_metrics_reads_total", gpu=0, kind="fresh")
    cpu = promtext.value(fams, "gpuexp_gpu_metrics_fetch_cpu_seconds_total", gpu=0)
    per_read_us = cpu / fresh * 1e6
    print(f"ticks {st['ticks']}, parts per tick (us): "
          f"{ {k: round(v / st['ticks'] * 1e6, 1) for k, v in parts.items()} }, fresh reads {fresh}, "
          f"fetch CPU {per_read_us:.1f} us per fresh read, stage CPU (us/tick): "
          f"{ {k: round(v / st['ticks'] / 1e3, 1) for k, v in st['stage_cpu_ns'].items()} }")
    assert fresh >= 10 and 20 <= per_read_us <= 2000, (fresh, per_read_us)
    assert parts["gpu_metrics"] >= 0.5 * sum(parts.values()), parts
    assert promtext.value(fams, "gpuexp_gpu_metrics_min_interval_seconds", gpu=0) == 0.0


def test_kfd_events_source_opens(native):
    """The KFD SMI event fd opens on the real GPU (AMDKFD_IOC_SMI_EVENTS) and the six
    per-GPU event counters are exported from the first tick."""
    e = amdsmi_engine(native, series_profile="full")
    try:
        e.tick()
        status = e.source_status()
        print(status)
        assert "kfd_events=on 1 GPU(s)" in status, status
        fams = promtext.parse(e.snapshot_text())
        ev = {s[1]["event"]: s[2] for s in promtext.samples(fams, "amd_gpu_kfd_events_total") if s[1]["gpu"] == "0"}
        assert set(ev) == {"vm_fault", "thermal_throttle", "gpu_pre_reset", "gpu_post_reset", "queue_eviction",
                           "queue_restore"}, ev
        assert all(v >= 0 for v in ev.values())
        up = [s[2] for s in promtext.samples(fams, "gpuexp_source_up") if s[1]["source"] == "kfd_events"]
        assert up == [1]
    finally:
        e.stop()


def test_full_profile_gtt_and_bad_pages(native):
    """GTT used/total from mem_info_gtt_*, board identity and loaded firmware versions, and,
    where the RAS bad-page table is readable, the retired HBM pages by state (a healthy
    board: none unreservable)."""
    e = amdsmi_engine(native, series_profile="full")
    try:
        e.tick()
        fams = promtext.parse(e.snapshot_text())
        total = promtext.value(fams, "amd_gpu_gtt_total_bytes", gpu=0)
        used = promtext.value(fams, "amd_gpu_gtt_used_bytes", gpu=0)
        print("GTT used/total:", used, total)
        assert total > 1 << 30 and 0 <= used <= total
        board = [lab for _, lab, _ in promtext.samples(fams, "amd_gpu_board_info") if lab["gpu"] == "0"]
        fw = {lab["component"]: lab["version"] for _, lab, _ in promtext.samples(fams, "amd_gpu_firmware_info")
              if lab["gpu"] == "0"}
        drv = [lab for _, lab, _ in promtext.samples(fams, "amd_driver_info")]
        print("board:", board, "\nfirmware:", fw, "\ndriver:", drv)
        assert board and board[0]["vbios_version"], board
        assert len(fw) >= 3 and all(v.startswith("0x") for v in fw.values()), fw
        assert drv and drv[0]["kernel"], drv
        pages = {s[1]["state"]: s[2] for s in promtext.samples(fams, "amd_gpu_retired_pages") if s[1]["gpu"] == "0"}
        print("retired pages:", pages or "table not readable here")
        if pages:
            assert set(pages) == {"retired", "pending", "unreservable"} and pages["unreservable"] == 0, pages
    finally:
        e.stop()


def test_xgmi_links_carry_amdsmi_peers(native):
    """Per-link xGMI series: each link's peer_bdf and byte counters agree with amdsmi's own
    link metrics (amdsmi_get_link_metrics) for the same link, the peers are distinct other
    GPUs of this host, and the accumulators do not run backwards."""
    amdsmi = pytest.importorskip("amdsmi")
    e = amdsmi_engine(native, series_profile="full")
    try:
        e.tick()
        f1 = promtext.parse(e.snapshot_text())
        amdsmi.amdsmi_init()
        try:
            h = amdsmi.amdsmi_get_processor_handles()[0]
            lm = amdsmi.amdsmi_get_link_metrics(h)
        finally:
            amdsmi.amdsmi_shut_down()
        time.sleep(0.2)
        e.tick()
        f2 = promtext.parse(e.snapshot_text())
    finally:
        e.stop()
    own = promtext.samples(f1, "amd_gpu_info")[0][1]["bdf"].lower()
    links = {s[1]["link"]: (s[1]["peer_bdf"].lower(), s[2]) for s in promtext.samples(f1, "amd_gpu_xgmi_read_bytes_total")
             if s[1]["gpu"] == "0"}
    later = {s[1]["link"]: s[2] for s in promtext.samples(f2, "amd_gpu_xgmi_read_bytes_total") if s[1]["gpu"] == "0"}
    print("links:", links)
    print("amdsmi link metrics:", lm)
    peers = [p for p, _ in links.values() if p]
    assert peers, links
    # every link that carries bytes names its peer (the 7 of an 8-GPU MI355X mesh)
    assert all(p for p, v in links.values() if v > 0), links
    assert len(set(peers)) == len(peers) and own not in peers, (own, peers)
    for p in peers:
        assert os.path.isdir(f"/sys/bus/pci/devices/{p}"), p  # a real PCI function of this host
    for k, (_, v) in links.items():
        assert later[k] >= v, (k, v, later[k])
    # amdsmi's per-link KB, read between our two ticks, lies between our two readings of the
    # link it names: the link index <-> peer association is amdsmi's own
    t1 = {p: v / 1024 for p, v in links.values() if p}
    t2 = {links[k][0]: later[k] / 1024 for k in links if links[k][0]}
    checked = 0
    for l in lm.get("links", []):
        bdf = str(l.get("bdf", "")).lower()
        if bdf in t1 and isinstance(l.get("read"), int):
            assert t1[bdf] <= l["read"] <= t2[bdf], (bdf, t1[bdf], l["read"], t2[bdf])
            checked += 1
    print("links checked against amdsmi:", checked)
    # amdgpu's own port map (what the sysfs-only backend uses): slot l of amdsmi's link list
    # is source port l of xgmi_port_num
    sys_peers = native.xgmi_peers_from_sysfs("", own)
    print("sysfs port map:", sys_peers)
    smi = [str(l.get("bdf", "")).lower() for l in lm.get("links", [])]
    for l, b in enumerate(smi[:8]):
        if b and not b.startswith("ffff"):
            assert sys_peers[l] == b, (l, b, sys_peers)


def test_units_are_physically_consistent(native):
    """End-to-end units: the energy counter's rate over 2 s matches the mean of the power
    gauge sampled at 10 Hz (J vs W), VRAM used matches amdsmi's own VRAM usage, and the
    throttle residencies are percentages."""
    amdsmi = pytest.importorskip("amdsmi")
    e = amdsmi_engine(native, series_profile="full")
    try:
        powers, t0 = [], None
        for k in range(21):
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            if k == 0:
                t0, e0 = time.monotonic(), promtext.value(fams, "amd_gpu_energy_joules_total", gpu=0)
            powers.append(promtext.value(fams, "amd_gpu_power_watts", gpu=0))
            time.sleep(0.1)
        t1, e1 = time.monotonic(), promtext.value(fams, "amd_gpu_energy_joules_total", gpu=0)
        vram = promtext.value(fams, "amd_gpu_vram_used_bytes", gpu=0)
        cap = promtext.value(fams, "amd_gpu_power_cap_watts", gpu=0)
        clk = {s[1]["clock"]: s[2] for s in promtext.samples(fams, "amd_gpu_clock_hz") if s[1]["gpu"] == "0"}
        thr = [s[2] for s in promtext.samples(fams, "amd_gpu_throttle_residency_percent") if s[1]["gpu"] == "0"]
        amdsmi.amdsmi_init()
        try:
            h = amdsmi.amdsmi_get_processor_handles()[0]
            usage = amdsmi.amdsmi_get_gpu_vram_usage(h)
            smi_clk = {}
            for name in ("GFX", "MEM", "SOC"):
                try:
                    smi_clk[name.lower()] = amdsmi.amdsmi_get_clock_info(h, getattr(amdsmi.AmdSmiClkType, name))
                except Exception as ex:  # noqa: BLE001
                    smi_clk[name.lower()] = str(ex)
        finally:
            amdsmi.amdsmi_shut_down()
    finally:
        e.stop()
    rate = (e1 - e0) / (t1 - t0)
    mean_p = sum(powers) / len(powers)
    print(f"energy rate {rate:.1f} W vs mean power gauge {mean_p:.1f} W; vram {vram / 2**20:.0f} MiB vs amdsmi {usage}")
    assert 0.75 * mean_p < rate < 1.25 * mean_p, (rate, mean_p)
    used_mb = usage.get("vram_used") if isinstance(usage, dict) else None
    if isinstance(used_mb, (int, float)):
        assert abs(vram / 2**20 - used_mb) < max(256, 0.02 * used_mb), (vram, used_mb)
    assert all(0 <= v <= 100 for v in thr), thr
    print("power cap", cap, "W; clocks", clk, "\namdsmi clock info:", smi_clk)
    for name, info in smi_clk.items():
        if isinstance(info, dict) and isinstance(info.get("clk"), (int, float)) and name in clk:
            mhz = clk[name] / 1e6
            assert abs(mhz - info["clk"]) <= max(150, 0.25 * info["clk"]), (name, mhz, info)
    assert 300 < cap < 2500 and max(powers) <= 1.1 * cap, (cap, max(powers))
    assert 0 < clk.get("gfx", 0) <= 3.0e9 and 0.5e9 < clk.get("mem", 0) < 3.0e9, clk


def test_xcc_busy_agrees_with_gfx_activity_under_gemm(native):
    """Per-XCD busy (the exporter's own gfx_busy_acc deltas) against the PMFW's
    average_gfx_activity while a GEMM pod saturates the GPU: both near 100 %, and their
    means within 15 points of each other; the gauges stay in 0-100."""
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r);"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, 8.0, 4), flush=True)" % ROOT],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    e = amdsmi_engine(native, series_profile="full")
    try:
        # the burn is up once its waves show in KFD (a fresh box's first imports take seconds)
        t0 = time.time()
        while time.time() - t0 < 60 and child.poll() is None:
            e.tick()
            if promtext.value(promtext.parse(e.snapshot_text()), "amd_gpu_cu_occupancy", gpu=0) > 0:
                break
            time.sleep(0.2)
        time.sleep(0.5)
        gfx, xcc, cu = [], [], []
        for _ in range(15):
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            gfx.append(promtext.value(fams, "amd_gpu_gfx_activity_percent", gpu=0))
            xcc.extend(s[2] for s in promtext.samples(fams, "amd_gpu_xcc_busy_percent") if s[1]["gpu"] == "0")
            cu.append(promtext.value(fams, "amd_gpu_cu_occupancy", gpu=0))
            time.sleep(0.1)
    finally:
        e.stop()
        out, _ = child.communicate(timeout=60)
    print("gemm:", out.strip()[-300:])
    mg, mx = sum(gfx) / len(gfx), sum(xcc) / max(1, len(xcc))
    print(f"gfx_activity mean {mg:.1f} %, per-XCD busy mean {mx:.1f} % over {len(xcc)} samples; "
          f"occupied CUs {sorted(cu)}")
    # KFD cu_occupancy = resident waves / max waves per CU ("CU-equivalents"): the 256x256
    # GEMM, 100 % busy on every XCD, reads 64 of 256 (measured).  KFD's per-process read
    # comes back 0 on some ticks of a continuously busy GPU (measured: 10 of 15 on one box,
    # 0 of 15 on others), so only its range and that it saw the waves at all are asserted.
    assert 0 < max(cu) <= 256 and min(cu) >= 0, cu
    assert xcc and all(0 <= v <= 100.5 for v in xcc), xcc
    assert mg > 60 and mx > 60, (mg, mx)
    assert abs(mg - mx) < 15, (mg, mx)


def test_pod_energy_tracks_gpu_energy(native):
    """A GEMM pod alone on the GPU (owner inferred from its process): its
    amd_pod_gpu_energy_joules_total grows by the GPU's own energy-counter delta."""
    from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r);"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, 6.0, 4), flush=True)" % ROOT],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    e = amdsmi_engine(native)
    try:
        pid, deadline = None, time.time() + 20
        while pid is None and time.time() < deadline:
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            big = [int(lab["pid"]) for _, lab, v in promtext.samples(fams, "amd_gpu_process_vram_bytes")
                   if v > 256 * (1 << 20)]
            pid = big[0] if big else None
            time.sleep(0.2)
        assert pid, "GEMM child not found"
        uid, cid = "0e0e0e0e-0000-4000-8000-000000000001", "ef" * 32
        e.set_pods([{"uid": uid, "namespace": "ml", "name": "gemm", "containers": {cid: "main"}}])
        e.set_pid_cgroup(pid, kubepods_cgroup(uid, cid))
        for _ in range(3):
            e.tick()
            time.sleep(0.1)

        def both():
            e.tick()
            f = promtext.parse(e.snapshot_text())
            pod = [s[2] for s in promtext.samples(f, "amd_pod_gpu_energy_joules_total") if s[1]["pod"] == "gemm"]
            return (pod[0] if pod else 0.0), promtext.value(f, "amd_gpu_energy_joules_total", gpu=0)
        p0, g0 = both()
        for _ in range(20):
            time.sleep(0.1)
            e.tick()
        p1, g1 = both()
    finally:
        e.stop()
        child.communicate(timeout=60)
    print(f"pod energy +{p1 - p0:.1f} J, GPU energy +{g1 - g0:.1f} J")
    assert g1 - g0 > 100  # a busy MI355X over ~2 s
    assert abs((p1 - p0) - (g1 - g0)) <= 0.02 * (g1 - g0), (p1 - p0, g1 - g0)


def test_pod_energy_survives_exporter_restart(native, tmp_path):
    """Checkpoint/resume on silicon: a GEMM pod's energy total is written to the state file
    when the exporter stops, comes back in the next exporter before the pod list does, and
    keeps growing from there (no counter reset for Prometheus to see)."""
    from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup
    state = str(tmp_path / "state")
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r);"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, 8.0, 4), flush=True)" % ROOT],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    uid, cid = "0e0e0e0e-0000-4000-8000-000000000002", "cd" * 32
    pods = [{"uid": uid, "namespace": "ml", "name": "gemm", "containers": {cid: "main"}}]

    def pod_energy(e):
        f = promtext.parse(e.snapshot_text())
        v = [s[2] for s in promtext.samples(f, "amd_pod_gpu_energy_joules_total") if s[1]["pod"] == "gemm"]
        return v[0] if v else None

    a = b = None
    try:
        a = amdsmi_engine(native, state_file=state)
        pid, deadline = None, time.time() + 20
        while pid is None and time.time() < deadline:
            a.tick()
            fams = promtext.parse(a.snapshot_text())
            big = [int(lab["pid"]) for _, lab, v in promtext.samples(fams, "amd_gpu_process_vram_bytes")
                   if v > 256 * (1 << 20)]
            pid = big[0] if big else None
            time.sleep(0.2)
        assert pid, "GEMM child not found"
        a.set_pods(pods)
        a.set_pid_cgroup(pid, kubepods_cgroup(uid, cid))
        for _ in range(15):
            a.tick()
            time.sleep(0.1)
        e1 = pod_energy(a)
        a.stop()  # final checkpoint
        a = None
        assert e1 and e1 > 50, e1
        b = amdsmi_engine(native, state_file=state)
        assert "restored" in b.source_status(), b.source_status()
        b.tick()
        e2 = pod_energy(b)  # before any pod list: the restored total, unchanged
        b.set_pods(pods)
        b.set_pid_cgroup(pid, kubepods_cgroup(uid, cid))
        for _ in range(15):
            b.tick()
            time.sleep(0.1)
        e3 = pod_energy(b)
    finally:
        for e in (a, b):
            if e is not None:
                e.stop()
        child.communicate(timeout=60)
    print(f"pod energy: {e1:.1f} J at stop, {e2:.1f} J restored, {e3:.1f} J after 1.5 s more")
    assert e2 == pytest.approx(e1, rel=1e-9)
    assert e3 > e2 + 50  # a busy MI355X draws hundreds of watts


_H2D = """
import json, sys, time, torch
src = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
dst = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
dst.copy_(src, non_blocking=True); torch.cuda.synchronize()
print("ready", flush=True)
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < 4.0:
    dst.copy_(src, non_blocking=True); torch.cuda.synchronize(); n += 1
print(json.dumps({"Bps": n * (1 << 30) / (time.perf_counter() - t0)}), flush=True)
"""


def test_pcie_bandwidth_under_host_to_device_copy(native):
    """amd_gpu_pcie_bandwidth_bytes_per_second (PMFW pcie_bandwidth_inst in Mb/s, / 8) while a
    child streams pinned host memory to the GPU at a measured payload rate: link traffic is
    the payload plus protocol overhead and the reverse direction's requests (measured
    1.15-1.22x), so between 1.0x and 1.4x.  (Read as the kernel header's GB/s it was
    ~9700x too high; profiles/provenance/tools/probe_pcie_units.py.)"""
    import json
    child = subprocess.Popen([sys.executable, "-c", _H2D], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             text=True)
    e = amdsmi_engine(native, kfd_detail_interval_s=0.0)
    vals, sdma = [], []
    try:
        assert "ready" in child.stdout.readline() or True
        time.sleep(0.5)
        for _ in range(25):
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            vals.append(promtext.value(fams, "amd_gpu_pcie_bandwidth_bytes_per_second", gpu=0))
            # the copying process (the one holding the 1 GiB device buffer): SDMA busy time
            big = [(v, lab["pid"]) for _, lab, v in promtext.samples(fams, "amd_gpu_process_vram_bytes")
                   if v > (1 << 30)]
            if big:
                pid = max(big)[1]
                sd = [v for _, lab, v in promtext.samples(fams, "amd_gpu_process_sdma_seconds_total")
                      if lab["pid"] == pid]
                if sd:
                    sdma.append((time.monotonic(), sd[0]))
            time.sleep(0.1)
    finally:
        e.stop()
        out, _ = child.communicate(timeout=60)
    line = [l for l in out.splitlines() if l.startswith("{")]
    assert line, out[-2000:]
    measured = json.loads(line[-1])["Bps"]
    vals.sort()
    med = vals[len(vals) // 2]
    print(f"H2D copy {measured / 1e9:.1f} GB/s; exporter PCIe bandwidth median {med / 1e9:.1f} GB/s "
          f"(min {vals[0] / 1e9:.1f}, max {vals[-1] / 1e9:.1f})")
    assert measured > 5e9
    assert 1.0 * measured < med < 1.4 * measured, (med, measured)
    if len(sdma) >= 2 and sdma[-1][0] > sdma[0][0]:
        rate = (sdma[-1][1] - sdma[0][1]) / (sdma[-1][0] - sdma[0][0])
        # HIP moves pinned host memory with blit kernels, not SDMA, on MI355X (measured: 0 s/s),
        # so this only shows the counter does not move without SDMA work
        print(f"copying process SDMA busy {rate:.2f} s/s")
        assert 0 <= rate < 16, rate


def test_kfd_events_real_queue_eviction():
    """A real KFD event end to end (tools/kfd_events_check.py): invalidating a host buffer
    registered with the GPU makes KFD evict and restore this process's queues; the engine
    (same process, so an unprivileged event client sees them) counts both on GPU 0 and
    attributes them to the process's pod."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kfd_events_check.py")], capture_output=True,
                       text=True, timeout=120)
    print(r.stdout[-3000:], r.stderr[-2000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "kfd events check produced no result"
    res = json.loads(line[-1][7:])
    assert res["moved"]["queue_eviction"] >= 1 and res["moved"]["queue_restore"] >= 1, res
    assert res["moved"]["vm_fault"] == 0 and res["moved"]["gpu_pre_reset"] == 0, res
    assert res["pod"].get("probe/evicted-pod/queue_eviction", 0) >= 1, res


@pytest.mark.parametrize("impl", ["hip", "queue"])
def test_sentinel_one_wave_per_xcd(native, impl):
    """Full profile: the sentinel run puts one wave on each XCD (placement read back from
    HW_REG_XCC_ID) and the PMFW reports each XCD's gfx clock — from the HIP plugin's own
    stream and from raw AQL dispatches on the PMC counters' queue alike."""
    kw = dict(enable_counters=True, counters_plugin=native.default_rocprof_plugin(), sentinel_impl="queue") \
        if impl == "queue" else dict(sentinel_impl="hip")
    e = amdsmi_engine(native, enable_sentinel=True, series_profile="full", **kw)
    try:
        status = e.source_status()
        if impl == "queue" and "counters=unavailable" in status:
            pytest.skip("PMC queue unavailable on this box: " + status)
        assert ("hsa sentinel" if impl == "queue" else "hip sentinel") in status, status
        for _ in range(6):
            e.tick()
            time.sleep(0.05)
        fams = promtext.parse(e.snapshot_text())
        print(status)
    finally:
        e.stop()
    lat = {lab["xcc"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_sentinel_xcc_dispatch_latency_seconds")}
    clk = {lab["xcc"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_xcc_clock_hz")}
    print("per-XCD latency:", lat, "\nper-XCD clock:", clk)
    assert len(clk) == 8 and all(50e6 < v < 3.0e9 for v in clk.values()), clk
    assert sorted(lat) == sorted(clk), (lat, clk)  # every XCD got a wave
    first = promtext.value(fams, "amd_gpu_sentinel_dispatch_latency_seconds", gpu=0)
    assert all(0 <= v < 0.5 for v in lat.values()) and 0 <= first < 0.5, (first, lat)
    # memory-latency probe: dependent uncached loads (~110 ns/hop idle on MI355X)
    hbm = promtext.value(fams, "amd_gpu_sentinel_memory_latency_seconds", gpu=0)
    xhbm = {lab["xcc"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_sentinel_xcc_memory_latency_seconds")}
    print("memory-chain load latency:", hbm, xhbm)
    assert 20e-9 < hbm < 50e-6, hbm
    assert sorted(xhbm) == sorted(clk), xhbm


@pytest.mark.parametrize("M,N,K,variant", [(128, 128, 64, 1), (256, 384, 512, 1), (1024, 1024, 1024, 1),
                                           (512, 2048, 4096, 1), (256, 256, 128, 2), (512, 768, 320, 2),
                                           (1024, 1024, 1024, 2), (2048, 256, 4096, 2)])
def test_gemm_bf16_numerics(native, on_gpu, M, N, K, variant):
    import torch
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, torch.cuda.current_stream().cuda_stream,
                        variant)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T  # fp32 reference of the same op
    err = (c.float() - ref).abs()
    # bf16 output rounding: |err| <= 2^-8 |ref| + accumulated fp32 noise
    assert (err <= 1e-2 * ref.abs() + 1e-2 * K ** 0.5).all(), err.max().item()


def test_gemm_identity_asymmetric(native, on_gpu):
    """A = I with asymmetric B catches transposed C writes (cdna_hip_programming.md §3)."""
    import torch
    M = N = 128
    K = 128
    a = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N * K, device="cuda", dtype=torch.float32).reshape(N, K) % 97).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, 0)
    torch.cuda.synchronize()
    assert torch.equal(c, b.T.contiguous())


def test_gemm_identity_asymmetric_256(native, on_gpu):
    """Same check through the 256x256 kernel's LDS-staged epilogue (every quadrant)."""
    import torch
    M = N = 512
    K = 512
    a = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N * K, device="cuda", dtype=torch.float32).reshape(N, K) % 97).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, 0, 2)
    torch.cuda.synchronize()
    assert torch.equal(c, b.T.contiguous())


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (768, 512, 320), (2048, 2048, 2048), (4096, 4096, 1024)])
def test_gemm_256_matches_128_bitwise_every_run(native, on_gpu, M, N, K):
    """Both kernels add the same fp32 MFMA partials in the same K order, so their outputs
    are bit-identical; repeating the pipelined kernel screens for LDS races (a tile read
    before its DMA landed or restaged while read shows up as a mismatch), incl. odd
    K-tile counts (K=320) that end the loop without a prefetch."""
    import torch
    torch.manual_seed(1)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), ref.data_ptr(), M, N, K, s, 1)
    for variant in (2, 3, 4, 5, 6, 7, 8):  # tile orders, priority forms, snake-B reads, ping-pong
        for _ in range(4):
            c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, s, variant)
            torch.cuda.synchronize()
            assert torch.equal(c, ref), (variant, (c.float() - ref.float()).abs().max().item())


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (768, 512, 320), (2048, 2048, 2048), (4096, 4096, 1024)])
def test_gemm_4wave_kernel_every_run(native, on_gpu, M, N, K):
    """Variant 9 (4 waves of 128x128, v_mfma_f32_32x32x16_bf16): its MFMA shape sums K in
    16-deep steps, so it is checked against the fp32 reference of the same op rather than
    bit-for-bit against the 16x16x32 kernels; repeated runs must agree bit-for-bit (a tile
    read before its DMA landed, or restaged while read, shows up as a mismatch)."""
    import torch
    torch.manual_seed(2)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    s = torch.cuda.current_stream().cuda_stream
    ref = a.float() @ b.float().T
    first = None
    for _ in range(4):
        c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, s, 9)
        torch.cuda.synchronize()
        err = (c.float() - ref).abs()
        assert (err <= 1e-2 * ref.abs() + 1e-2 * K ** 0.5).all(), err.max().item()
        if first is None:
            first = c
        else:
            assert torch.equal(c, first)


def test_gemm_4wave_identity_asymmetric(native, on_gpu):
    """A = I with an asymmetric B through the 32x32x16 C layout and the LDS epilogue."""
    import torch
    M = N = K = 512
    a = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N * K, device="cuda", dtype=torch.float32).reshape(N, K) % 97).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    kernels().gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, 0, 9)
    torch.cuda.synchronize()
    assert torch.equal(c, b.T.contiguous())


def test_gemm_rejects_bad_shapes(native):
    with pytest.raises(ValueError):
        kernels().gemm_bf16(1, 1, 1, 100, 128, 64, 0)
    with pytest.raises(ValueError):  # 256x256 kernel: N % 256 and K >= 128
        kernels().gemm_bf16(1, 1, 1, 256, 384, 128, 0, 2)
    with pytest.raises(ValueError):
        kernels().gemm_bf16(1, 1, 1, 256, 256, 64, 0, 2)


def test_gemm_burn_throughput(native):
    r = kernels().gemm_burn(0, 4096, 4096, 4096, 1.0, 8)
    print("gemm 4096^3 bf16:", r)
    assert r["tflops"] > 100  # sanity: MFMA path, not a scalar fallback
    r1 = kernels().gemm_burn(0, 8192, 8192, 8192, 1.0, 4, 1)
    r2 = kernels().gemm_burn(0, 8192, 8192, 8192, 1.0, 4, 2)
    print("gemm 8192^3 bf16 TFLOP/s: 128x128", round(r1["tflops"]), "256x256", round(r2["tflops"]))
    assert r2["tflops"] > r1["tflops"]  # the default (256x256) kernel is the faster one


@pytest.mark.parametrize("nbytes,blocks", [(64 << 20, 4096), ((1 << 20) + 48, 7), (4096 * 16 * 256 + 16, 4096),
                                           (16, 1)])
def test_stream_copy_numerics(native, nbytes, blocks):
    """The calibration copy (probe_device.h, HIP launch) is an exact byte copy for chunk
    tails, uneven chunks and grids with more workgroups than vectors; the bytes outside
    the destination range stay untouched."""
    import torch
    from kubernetes_gpu_exporter_amd.ops.gemm import stream_copy
    g = torch.Generator(device="cuda").manual_seed(nbytes)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
    guard = torch.full((nbytes + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
    stream_copy(src, guard[:nbytes], blocks=blocks)
    torch.cuda.synchronize()
    assert torch.equal(guard[:nbytes], src)
    assert bool((guard[nbytes:] == 0xA5).all())


@pytest.mark.parametrize("conflicts", [False, True])
def test_lds_probe_numerics(native, conflicts):
    """lds_probe: lane 0 of each workgroup sums table[i mod 4096] = (i mod 4096) & 7 over
    `iters` reads (stride only moves the other lanes) — compared with the fp32 reference."""
    import torch
    from kubernetes_gpu_exporter_amd.ops.gemm import lds_probe
    blocks, iters = 300, 5000
    out = torch.zeros(blocks, dtype=torch.float32, device="cuda")
    lds_probe(out, blocks, iters, conflicts)
    torch.cuda.synchronize()
    ref = float(((torch.arange(iters) % 4096) & 7).to(torch.float32).sum())
    assert torch.equal(out.cpu(), torch.full((blocks,), ref))


def _feature_check(*args, timeout=300):
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gpu_features_check.py"), *args],
                       capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-3000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "feature check produced no result"
    return json.loads(line[-1][7:])


@pytest.mark.parametrize("plugin", ["aqlpmc", "rocprof"])
def test_device_counters_under_gemm(plugin, monkeypatch):
    """MFMA/GUI (+ LDS/HBM where the PMCs are device-scoped) counters while a GEMM pod runs
    (BASELINE config 4), from both counter plugins.  The aqlprofile plugin must not cost a
    core (the rocprofiler-sdk one does: see rocprof_plugin.cc).  Skips — loudly — when the
    box denies PMC access."""
    monkeypatch.setenv("PLUGIN", plugin)
    res = _feature_check("counters", "3")
    if "counters=unavailable" in res["status"]:
        pytest.skip("device counting unavailable on this box: " + res["status"])
    assert res["gemm_running_at_snapshot"], res
    assert res["amd_gpu_mfma_busy_percent"] is not None, res
    assert res["amd_gpu_mfma_busy_percent"] > 10, res   # an MFMA GEMM is running
    assert res["amd_gpu_gui_active_percent"] > 50, res
    if res["device_scope"] == 1:
        assert res["amd_gpu_hbm_read_bytes_per_second"] > 1e9, res
        assert res["series_gpu0"] == 64, res  # standard profile: the remote (GMI) pair is full-profile only
    else:  # wave/LDS/EA counters VMID-filtered to the exporter: not exported as device totals
        assert res["series_gpu0"] == 58, res
    if plugin == "aqlpmc":
        assert max(p for p, _ in res["hot_threads"]) < 20.0, res


def test_mfma_busy_calibration():
    """amd_gpu_mfma_busy_percent against kernels of known MFMA duty (tools/mfma_calibration.py):
    the engine at 10 Hz with continuous counters while 2 waves per SIMD alternate
    back-to-back v_mfma_f32_32x32x16_bf16 with s_sleep at 25/50/75/100 % of the wall time.

    * every resident case reads within 10 points of its duty (the counter is cycle-weighted:
      the chip clocks down during the MFMA phases, so it reads a few points low), and
      changes every tick (continuous counting: each tick exports its own interval);
    * SQ_VALU_MFMA_BUSY_CYCLES over each kernel's life equals 32 cycles per MFMA the kernel
      counted itself issuing (MI355X_MICROARCH.md cycle constants) within 1 %;
    * gated cases (100 % MFMA kernels for 25 / 50 % of every 20 ms, idle between): busy =
      GUI-active x MfmaUtil, and MfmaUtil (while active) stays high;
    * an idle GPU reads 0."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_calibration.py"), "--duties",
                        "0.25,0.5,0.75,0.98"], capture_output=True, text=True, timeout=200)
    print(r.stdout[-4000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "calibration produced no result"
    res = json.loads(line[-1][7:])
    if "counters=unavailable" in res["status"]:
        pytest.skip("device counting unavailable on this box: " + res["status"])
    assert "continuous" in res["status"], res["status"]
    cases = res["cases"]
    assert cases["idle"]["busy_median"] == 0.0, cases["idle"]
    for key in ("resident_0.25", "resident_0.5", "resident_0.75", "resident_0.98"):
        c = cases[key]
        assert c["ticks"] >= 15, (key, c["ticks"])
        assert abs(c["busy_median"] - c["expected_busy"]) <= 10.0, (key, c["busy_median"], c["expected_busy"])
        assert c["changed_fraction"] >= 0.9, (key, c["per_tick_busy"])
        assert abs(c["mfma_busy_cycles_over_32x_issued"] - 1.0) < 0.01, (key, c["mfma_busy_cycles_over_32x_issued"])
    for key in ("gated_0.5", "gated_0.25"):
        c = cases[key]
        assert c["util_median"] > 80, (key, c)
        assert abs(c["busy_median"] - c["gui_median"] * c["util_median"] / 100.0) < 5.0, (key, c)
        assert c["changed_fraction"] >= 0.9, (key, c["per_tick_busy"])


def test_xcc_mfma_busy_calibration():
    """amd_gpu_xcc_mfma_busy_percent against an MFMA kernel confined to one XCD: the duty
    kernel at 90 % whose blocks leave at once unless HW_REG_XCC_ID is the target.  That XCD
    reads within 10 points of 90, every other XCD reads ~0, and the chip value is the mean
    of the eight (each XCD's busy cycles over its own elapsed cycles).  Then 2 s of MFMAs on
    every SIMD: amd_gpu_sentinel_pending_seconds grows while the sentinel's run waits behind
    them and is 0 before and after, and the counter reads stuck behind that run move to a
    queue of their own, so MFMA busy stays exported (~100 %) through the starvation."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_calibration.py"), "--duties", "",
                        "--xcc-cases", "2,5", "--xcc-duty", "0.9", "--no-gated", "--starve", "2.0"],
                       capture_output=True, text=True, timeout=120)
    print(r.stdout[-4000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "calibration produced no result"
    res = json.loads(line[-1][7:])
    if "counters=unavailable" in res["status"]:
        pytest.skip("device counting unavailable on this box: " + res["status"])
    assert res["cases"]["idle"]["xcc_median"] == {str(x): 0.0 for x in range(8)}, res["cases"]["idle"]
    for x in (2, 5):
        c = res["cases"][f"xcc_{x}"]
        xs = c["xcc_median"]
        assert sorted(xs) == [str(i) for i in range(8)], xs
        assert abs(xs[str(x)] - 90.0) <= 10.0, (x, xs)
        assert all(v < 1.0 for k, v in xs.items() if k != str(x)), (x, xs)
        assert abs(c["busy_median"] - sum(xs.values()) / 8) < 0.5, (x, c["busy_median"], xs)
        assert c["waves_that_ran"] == c["waves"] // 8, c
    st = res["cases"]["starve"]
    # 2 s of MFMAs on every SIMD: the sentinel's run waits behind them, then completes
    assert st["pending_before"] == 0.0, st
    # (how long one run waits varies: the grid's blocks run in generations, and at a generation
    # change the dispatcher may place the sentinel's waves -- its longest wait ran 1.0 s in
    # round 6's sessions 9, 10 and 12, 0.5 s in session 13, each of them reset and launched again 0.5 s later;
    # 0.25 s = held behind the grid for two ticks and more after its launch)
    assert st["pending_max"] >= 0.25, st
    assert st["pending_after"] == 0.0, st
    # the counter reads held behind that run moved to a queue of their own (read rescue):
    # MFMA busy kept being exported through the starvation, near 100 %
    assert st["rescued"] == "1", st
    # ... temporarily: once the first queue drains, reads return there and the rescue queue
    # (its 173 MiB context save area) is released; the process's RSS returns to within
    # 10 MiB of where it was before the starvation
    assert st["rescue_active_after"] == "0" and st["rescues"] == st["rescue_releases"], st
    rss = st["rss_mib"]
    assert abs(rss["after"] - rss["before"]) <= 10.0, rss
    # ... and the self-metrics say so
    ev = st["counters_events"]
    assert ev.get("rescue", 0) >= 1 and ev.get("rescue_release", 0) == ev.get("rescue"), ev
    assert st["rescue_active_metric"] == 0.0, st
    during = st["busy_during"][8:]  # from 0.8 s on (3 stuck rounds + the move)
    assert sum(v is not None for v in during) >= 0.8 * len(during), st
    # near 100 % while the grid runs; the grid's blocks run in generations (every wave slot
    # is taken), so a window straddling a generation change may dip (one run: a 15 % sample)
    import statistics
    assert statistics.median(v for v in during if v is not None) > 80.0, st


def test_occupancy_limiters_see_other_processes():
    """Occupancy limiters as device-wide signals (SPI resource-allocator counters,
    amd_gpu_occupancy_limiter_percent / amd_gpu_dispatch_stall_percent), against kernels of
    known limiter run by ANOTHER process, four generations of blocks queued: 1 wave + 64 KiB
    of LDS per block -> LDS limits; 8 waves per block, no LDS -> wave slots; 1 wave of 400
    registers per lane -> VGPRs; 1 wave of 108 SGPRs -> SGPRs (7 of a SIMD's 8 slots fill
    first).  The dispatcher is stalled most of the time; idle: nothing waits (0).  Read from
    the engine's own exposition on an unprivileged box (profiles/r04/spi_scope.txt)."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_spi_scope.py"), "--seconds", "2.0",
                        "--no-self", "--exported", "--kinds", "lds,waves,vgpr,sgpr"],
                       capture_output=True, text=True, timeout=200)
    print(r.stdout[-3000:], r.stderr[-2000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "probe produced no result"
    res = json.loads(line[-1][7:])
    if "counters=unavailable" in res["status"]:
        pytest.skip("device counting unavailable on this box: " + res["status"])
    cases = res["cases"]
    idle = cases["idle"]["exported_median"]
    assert idle["stall"] == 0.0 and idle["lds"] == 0.0, idle
    others = {"lds", "wave_slots", "vgpr", "sgpr"}
    for case, limiter, stall in (("lds_other", "lds", 90), ("waves_other", "wave_slots", 90),
                                 ("vgpr_other", "vgpr", 90), ("sgpr_other", "sgpr", 50)):
        m = cases[case]["exported_median"]
        assert m["stall"] > stall and m[limiter] > 90, (case, m)
        # the LDS kernel's waves also leave 2 of 4 SIMDs without VGPRs for the next (vgpr ~50)
        assert all(m[o] < 5 for o in others - {limiter} - ({"vgpr"} if case == "lds_other" else set())), (case, m)


def test_device_scope_pmc_calibration():
    """Device-scope PMC families against ground truth (tools/pmc_validate.py): HBM read and
    write of a stream copy of known bytes, waves/s of known grids, LDS bank conflicts of a
    conflict-free vs a 32-way-conflicted read pattern, and MFMA FLOP/s by operand type of a
    known number of bf16 / fp8 MFMAs.  The workloads run on the PMC
    queue itself (the only queue an unprivileged process's SQ/TCC counters see)."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_validate.py")], capture_output=True,
                       text=True, timeout=240)
    print(r.stdout[-4000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
    assert line, "calibration produced no result"
    res = json.loads(line[-1][7:])
    if "counters=unavailable" in res["status"]:
        pytest.skip("device counting unavailable on this box: " + res["status"])
    cp, clean, conf = res["copy"], res["lds_clean"], res["lds_32way"]
    for w in (cp, clean, conf):  # each read window lies inside its workload's busy period
        assert w.get("busy_at_tick", True), w
    assert cp["device_scope"] == 1, cp
    rd = cp["amd_gpu_hbm_read_bytes_per_second"] / cp["expected_Bps"]
    wr = cp["amd_gpu_hbm_write_bytes_per_second"] / cp["expected_Bps"]
    print(f"HBM read {rd:.3f}x, write {wr:.3f}x of the copy's bytes/s")
    assert 0.9 < rd < 1.1 and 0.9 < wr < 1.1, (rd, wr)
    # the PMFW's UMC-activity estimate (amd_gpu_hbm_bandwidth_bytes_per_second, device-wide,
    # no PMC needed) against the copy's read + write bytes
    est = cp["amd_gpu_hbm_bandwidth_bytes_per_second"] / (2 * cp["expected_Bps"])
    print(f"UMC-activity HBM estimate {est:.3f}x of the copy's read+write bytes/s")
    assert 0.85 < est < 1.15, est
    # a local copy sends nothing to memory behind GMI (peer GPUs)
    assert cp["amd_gpu_remote_read_bytes_per_second"] < 0.01 * cp["expected_Bps"], cp
    assert cp["amd_gpu_remote_write_bytes_per_second"] < 0.01 * cp["expected_Bps"], cp
    for w in (cp, clean, conf):
        ratio = w["amd_gpu_waves_per_second"] / w["expected_waves_per_second"]
        assert 0.9 < ratio < 1.1, (ratio, w)
    assert clean["amd_gpu_lds_active_percent"] > 0 and conf["amd_gpu_lds_active_percent"] > 0
    assert clean["amd_gpu_lds_bank_conflict_percent"] < 10, clean
    # 32-way: 31 of every 32 LDS cycles are conflict cycles (96.875 %)
    assert abs(conf["amd_gpu_lds_bank_conflict_percent"] - 100 * 31 / 32) < 2, conf
    # MFMA FLOP/s by operand type against a fixed count of 32x32x16 MFMAs per wave
    # (measured 1.0004x bf16, 0.9997x fp8: profiles/r03/mfma_flops_calibration.txt)
    for name, dtype, other in (("mfma_bf16", "bf16", "fp8"), ("mfma_fp8", "fp8", "bf16")):
        w = res[name]
        assert w.get("busy_at_tick", True) and "expected_flops_per_second" in w, w
        ratio = w["flops_" + dtype] / w["expected_flops_per_second"]
        print(f"{dtype} MFMA FLOP/s {ratio:.4f}x of the issued work")
        assert 0.97 < ratio < 1.03, (name, ratio, w)
        assert w["flops_" + other] < 0.01 * w["expected_flops_per_second"], (name, w)


def test_rccl_tracer_counts_collectives():
    res = _feature_check("rccl")
    assert res["rc"] == 0, res
    assert res["files"], res
    ops = res["ops"]
    assert ops["allreduce"]["calls"] >= 20
    assert ops["allreduce"]["bytes"] >= 20 * (2 << 20)
    assert ops["allgather"]["calls"] >= 5
    assert res["communicator"] == [{"rank": 0, "nranks": 1}], res["communicator"]  # ncclCommUserRank/Count
    assert ops["reducescatter"]["calls"] >= 5 and ops["alltoall"]["calls"] >= 5, ops
    # every strategy's traced calls and bytes == the generator's ground truth, byte for byte
    par = res["parity"]
    assert set(par) == {"dp", "tp", "sp", "ep", "ulysses", "bcast", "p2p"}, par
    # PP/CP point-to-point (grouped send+recv to self) and gather/scatter via RCCL's C API
    assert par["p2p"]["data_ok"] is True, par["p2p"]
    for strategy, p in par.items():
        assert p["traced"] == p["expected"], (strategy, p)


def test_process_discovery_under_workload(native):
    """A child GEMM process appears in the KFD process list with its VRAM and the GPU's
    gfx activity rises while it runs."""
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r);"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, 6.0, 4), flush=True)" % ROOT],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    e = amdsmi_engine(native)
    try:
        seen_pids = set()
        max_gfx = 0.0
        max_share = 0.0
        nsp = open("/proc/self/status").read().split("NSpid:")[1].split("\n")[0].split()
        print("NSpid of test process:", nsp, "child pid", child.pid)
        deadline = time.time() + 5
        while time.time() < deadline:
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            for _, lab, v in promtext.samples(fams, "amd_gpu_process_vram_bytes"):
                if v > 256 * (1 << 20):
                    seen_pids.add(int(lab["pid"]))
            big = {str(p) for p in seen_pids}
            for _, lab, v in promtext.samples(fams, "amd_gpu_process_gfx_activity_percent"):
                if lab["pid"] in big:
                    max_share = max(max_share, v)
            try:
                max_gfx = max(max_gfx, promtext.value(fams, "amd_gpu_gfx_activity_percent", gpu=0))
            except KeyError:
                pass
            time.sleep(0.2)
        print("processes with >256MiB VRAM:", seen_pids, "max gfx activity", max_gfx)
        print("kfd proc dir:", sorted(os.listdir("/sys/class/kfd/kfd/proc")))
        assert seen_pids, "GEMM child not found in KFD process list"
        assert max_gfx > 50
        # the GEMM holds (nearly) every occupied CU, so it gets (nearly) all the activity
        print("max gfx share of the GEMM process:", max_share)
        assert max_share > 40
        if len(nsp) == 1:
            assert child.pid in seen_pids or any(p != child.pid for p in seen_pids)
    finally:
        e.stop()
        out, _ = child.communicate(timeout=60)
        print("child:", out.strip())


def test_two_pods_share_one_gpu(native):
    """Two GEMM processes on one GPU (a shared GPU, no device-plugin owner): both appear
    with their VRAM, and the GPU's gfx activity is split between them by occupied CUs —
    the shares add up to the device activity on every tick."""
    code = ("import sys; sys.path.insert(0, %r);"
            "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
            "print(gemm_burn(0, 4096, 5.0, 4), flush=True)" % ROOT)
    kids = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             text=True) for _ in range(2)]
    e = amdsmi_engine(native, kfd_detail_interval_s=0.0)
    try:
        best: dict = {}
        sums_ok = ticks = 0
        deadline = time.time() + 4.5
        while time.time() < deadline:
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            vram = {lab["pid"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_process_vram_bytes")
                    if v > 256 * (1 << 20)}
            share = {lab["pid"]: v for _, lab, v in promtext.samples(fams, "amd_gpu_process_gfx_activity_percent")}
            if len(vram) >= 2:
                ticks += 1
                act = promtext.value(fams, "amd_gpu_gfx_activity_percent", gpu=0)
                if abs(sum(share.values()) - act) < 0.5:
                    sums_ok += 1
                for pid in vram:
                    best[pid] = max(best.get(pid, 0.0), share.get(pid, 0.0))
            time.sleep(0.2)
        print("ticks with both:", ticks, "sum==activity:", sums_ok, "max share per pid:", best)
        assert ticks >= 3, "the two GEMM processes were not both visible"
        assert sums_ok == ticks
        assert len([p for p, v in best.items() if v > 5]) >= 2, best
    finally:
        e.stop()
        for k in kids:
            print("child:", k.communicate(timeout=60)[0].strip()[-200:])


def test_gemm_pod_model_on_gpu(native):
    """models.GemmPod runs the HIP kernel (not a torch fallback) and matches fp32."""
    import torch
    from kubernetes_gpu_exporter_amd.models import GemmPod, run
    p = GemmPod(size=512, iters=1)
    assert p.gpu and p.c.dtype == torch.bfloat16
    p.step()
    ref = p.a.float() @ p.b.float().T
    torch.testing.assert_close(p.c.float(), ref, atol=0.05, rtol=0.02)
    big = run(GemmPod(size=4096, iters=8), steps=3, warmup=1)
    assert big["tflops"] > 100, big


def test_raw_metrics_path_and_pmfw_coalescing(native):
    """The amdsmi backend reads gpu_metrics raw (no silent library fallback) and, at
    100 Hz, learns the ~20 ms PMFW refresh and skips the SMU fetch in between.  The CPU cap of
    the auto fetch policy is off here (metrics_min_interval_s = 0): at round 6's 0.75 % budget
    it alone would fetch every 4th 10 ms tick, and the refresh period is only learnt from
    fresh reads on consecutive ticks (it read 0.0 in profiles/r06/session2/pytest_gpu.log)."""
    c = native.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.01
    c.metrics_min_interval_s = 0
    c.serve_http = False
    c.device_filter = [0]
    e = native.Engine(c)
    e.start()
    time.sleep(2.0)
    fams = promtext.parse(e.snapshot_text())
    status = e.source_status()
    e.stop()
    assert "raw gpu_metrics v1.8 (validated against amdsmi: " in status, status
    reads = {s[1]["kind"]: s[2] for s in promtext.samples(fams, "gpuexp_gpu_metrics_reads_total")}
    frac = reads["coalesced"] / (reads["fresh"] + reads["coalesced"])
    # ~half at 100 Hz vs a 20 ms PMFW refresh (0.62 seen when a refresh lands just after a
    # tick and the next fresh read waits one more tick); never all of them
    assert 0.3 < frac < 0.75, reads
    (period,) = [s[2] for s in promtext.samples(fams, "gpuexp_gpu_metrics_refresh_period_seconds")]
    # ~20 ms on most boxes; one idle box's firmware stepped every 30.0 ms (learnt 0.0300036 s):
    # the learnt value follows the firmware, so accept anything up to the reuse cap (50 ms)
    assert 0.015 < period < 0.05, period
    # fresh reads track the refresh rate, not the tick rate: at most one per refresh period
    assert reads["fresh"] * period < 2.0 * 1.5, (reads, period)


def test_hip_order_bdfs_match_torch():
    """bench.py watches the ranks' GPUs by BDF computed without initialising HIP; it must
    agree with HIP's own device order."""
    import torch
    from kubernetes_gpu_exporter_amd.utils.kfdself import hip_order_bdfs
    bdfs = hip_order_bdfs()
    assert len(bdfs) == torch.cuda.device_count(), bdfs
    for i, b in enumerate(bdfs):
        p = torch.cuda.get_device_properties(i)
        dom = getattr(p, "pci_domain_id", 0)
        assert b == f"{dom:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0", (i, b)


def test_rccl_tracer_through_exporter(native, tmp_path):
    """End to end on silicon: a tracer-injected RCCL process writes its counters file and
    the exporter's RCCL source proves the writer (PID namespace, /proc/<pid>/maps of the
    file, pidfd) and exports its calls and bytes under that PID while it runs."""
    from kubernetes_gpu_exporter_amd._native import rccl_tracer_path
    d = str(tmp_path)
    import socket
    with socket.socket() as s:  # a free port for the child's TCP store
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, ROCP_TOOL_LIBRARIES=rccl_tracer_path(), GPUEXP_RCCL_DIR=d,
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    code = ("import time, torch, torch.distributed as dist\n"
            "dist.init_process_group('nccl', rank=0, world_size=1)\n"
            "torch.cuda.set_device(0)\n"
            "x = torch.ones(1 << 20, device='cuda', dtype=torch.bfloat16)\n"
            "t = time.time()\n"
            "while time.time() - t < 6:\n"
            "    dist.all_reduce(x); torch.cuda.synchronize(); time.sleep(0.01)\n"
            "dist.destroy_process_group()\n")
    child = subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True)
    e = amdsmi_engine(native, enable_rccl=True, rccl_dir=d, series_profile="full")
    try:
        calls, files, listing = 0.0, {}, []
        deadline = time.time() + 60
        while time.time() < deadline and child.poll() is None:
            e.tick()
            fams = promtext.parse(e.snapshot_text())
            files = {lab["state"]: v for _, lab, v in promtext.samples(fams, "gpuexp_rccl_files")}
            for _, lab, v in promtext.samples(fams, "amd_rccl_collective_calls_total"):
                if lab["op"] == "allreduce":
                    calls = max(calls, v)
                    pid = int(lab["pid"])
            listing = os.listdir(d)
            if calls >= 10:
                break
            time.sleep(0.2)
        print("tracer files:", listing, "states:", files, "allreduce calls:", calls)
        assert calls >= 10, (listing, files, e.source_status())
        assert files.get("active") == 1, files
        assert pid == child.pid or len(open("/proc/self/status").read().split("NSpid:")[1].split("\n")[0].split()) > 1
    finally:
        e.stop()
        out, _ = child.communicate(timeout=60)
        print("child:", out.strip()[-500:])


def test_compiled_exposition_on_silicon(native):
    """The fixed-layout exposition with real telemetry (full profile, sentinel, counters): a
    gzip scraper at the tick rate gets members that inflate (zlib, an independent inflater) to
    text parsing to the same families and series as the identity body, and once the layout has
    settled the body stops being laid out again and its gzip stays small (session 6 of round 5
    had 22-32 KB for a 49 KB body while one settle clock kept families provisional)."""
    import gzip
    c = native.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.05
    c.device_filter = [0]
    c.series_profile = "full"
    c.enable_sentinel = True
    c.serve_http = True
    h = c.http
    h.port = 0
    h.host = "127.0.0.1"
    c.http = h
    e = native.Engine(c)
    e.start()
    try:
        gz = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", True, 5000)
        ident = native.ScrapeClient("127.0.0.1", e.http_port, "/metrics", False, 5000)
        t_ready = time.time() + 10.0  # 503 until the first tick published (device open, first reads)
        while ident.scrape() <= 0 or ident.last_status != 200:
            assert time.time() < t_ready, ident.last_status
            time.sleep(0.05)
        t_end = time.time() + 3.0
        while time.time() < t_end:  # 20 Hz gzip asks, as Prometheus would at this rate
            assert gz.scrape() > 0 and gz.last_status == 200
            time.sleep(0.05)
        s0 = e.stats()
        sizes = []
        for _ in range(20):
            assert gz.scrape() > 0 and ident.scrape() > 0
            text = gzip.decompress(gz.last_body()).decode()
            body = ident.last_body().decode()
            a, b = promtext.parse(text), promtext.parse(body)
            assert a.keys() == b.keys()
            for name in a:  # the same series (values may differ by a tick)
                assert sorted(sorted(lab.items()) for _, lab, _ in a[name].samples) == \
                    sorted(sorted(lab.items()) for _, lab, _ in b[name].samples), name
            sizes.append((len(gz.last_body()), len(text)))
            time.sleep(0.05)
        s1 = e.stats()
    finally:
        e.stop()
    relayouts = s1["relayouts"] - s0["relayouts"]
    ratio = max(g / t for g, t in sizes)
    print(f"gzip / text: {sizes[-1]}, worst ratio {ratio:.3f}; relayouts over the last "
          f"{s1['ticks'] - s0['ticks']} ticks: {relayouts}; code builds {s1['code_builds']}")
    assert ratio < 0.35, sizes
    assert relayouts <= 3, relayouts
