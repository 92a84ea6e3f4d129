"""Engine on the mock backend (BASELINE config 1): series profile, legacy-family
compatibility, rates from hardware accumulators, fault isolation, attribution."""
import collections

import pytest

from kubernetes_gpu_exporter_amd.utils import promtext
from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup

S = 1_000_000_000
UID = "12345678-1234-1234-1234-123456789abc"
CID = "a" * 64
CG = ("/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod"
      + UID.replace("-", "_") + ".slice/cri-containerd-" + CID + ".scope")


def ticks(e, n, t0=S, dt=S // 10):
    t = t0
    for _ in range(n):
        e.tick(t)
        t += dt
    return t


def parse(e):
    return promtext.parse(e.snapshot_text())


def device_series_per_gpu(fams):
    cnt = collections.Counter()
    for name, fam in fams.items():
        if not name.startswith("amd_gpu_") or name.startswith("amd_gpu_process_"):
            continue
        for _, labels, _ in fam.samples:
            cnt[labels["gpu"]] += 1
    return cnt


@pytest.mark.parametrize("n", [1, 2, 8])
def test_standard_profile_is_64_series_per_gpu(mock_engine, n):
    e = mock_engine(n, http=False, enable_sentinel=True, enable_counters=True)
    ticks(e, 3)
    cnt = device_series_per_gpu(parse(e))
    assert dict(cnt) == {str(i): 64 for i in range(n)}


def test_compact_and_legacy_profiles(mock_engine):
    e = mock_engine(1, http=False, series_profile="compact")
    ticks(e, 3)
    assert device_series_per_gpu(parse(e))["0"] < 40
    e2 = mock_engine(1, http=False, series_profile="legacy")
    e2.mock_set_processes(0, [dict(pid=100, vram_bytes=1e9)])
    e2.set_pid_cgroup(100, CG)
    e2.set_pods([dict(uid=UID, namespace="ml", name="trainer-0", containers={})])
    ticks(e2, 2)
    fams = parse(e2)
    assert not [n for n in fams if n.startswith("amd_")]
    assert "pod_gpu_memory_usage" in fams


@pytest.mark.parametrize("exposition", ["classic", "compiled"])
def test_legacy_families_exact_contract(mock_engine, exposition):
    """Names, HELP, TYPE and label order byte-identical to /root/reference/main.go:22-35.  The
    compiled exposition blank-pads values to a fixed width (text parsers skip blanks after a
    value); the classic one writes them bare, byte for byte as client_golang does."""
    import re
    e = mock_engine(1, http=False, exposition=exposition)
    e.mock_set_processes(0, [dict(pid=4242, vram_bytes=30922086809.6)])
    e.set_pid_cgroup(4242, CG)
    e.set_pods([dict(uid=UID, namespace="ml", name="trainer-0", containers={CID: "main"})])
    ticks(e, 2)
    text = e.snapshot_text()
    pad = "" if exposition == "classic" else " *"  # compiled: the value right-aligned behind blanks
    assert re.search(re.escape("# HELP docker_gpu_memory_perc_usage GPU memory in percentage used by pod\n"
                               "# TYPE docker_gpu_memory_perc_usage gauge\n"
                               'docker_gpu_memory_perc_usage{pid="4242",pod="trainer-0"} ') + pad +
                     re.escape("10\n"), text)
    assert re.search(re.escape("# HELP pod_gpu_memory_usage GPU memory used by Kubernetes Pod\n"
                               "# TYPE pod_gpu_memory_usage gauge\n"
                               'pod_gpu_memory_usage{pid="4242",pod="trainer-0"} ') + pad +
                     re.escape("30922086809.6\n"), text)
    # docker_ sorts before pod_ (client_golang Gather order)
    assert text.index("docker_gpu_memory_perc_usage") < text.index("pod_gpu_memory_usage")


def test_legacy_sums_over_gpus_and_skips_unattributed(mock_engine):
    e = mock_engine(2, http=False)
    e.mock_set_processes(0, [dict(pid=10, vram_bytes=100.0), dict(pid=11, vram_bytes=5.0)])
    e.mock_set_processes(1, [dict(pid=10, vram_bytes=300.0)])
    e.set_pid_cgroup(10, CG)  # pid 11 has no pod
    e.set_pods([dict(uid=UID, namespace="ml", name="trainer-0", containers={})])
    ticks(e, 2)
    fams = parse(e)
    assert promtext.value(fams, "pod_gpu_memory_usage", pid=10) == 400.0
    pct = promtext.value(fams, "docker_gpu_memory_perc_usage", pid=10)
    assert abs(pct - 400.0 / (2 * 309220868096) * 100) < 1e-12
    with pytest.raises(KeyError):
        promtext.value(fams, "pod_gpu_memory_usage", pid=11)
    # the new per-process family keeps unattributed processes (pod="")
    assert promtext.value(fams, "amd_gpu_process_vram_bytes", pid=11, pod="") == 5.0
    assert promtext.value(fams, "pod_gpu_memory_usage", pid=10, pod="trainer-0") == 400.0
    # pod name unknown to the control plane -> no legacy series (never the UID as `pod`)
    e.set_pods([])
    ticks(e, 2, t0=10 * S)
    fams = parse(e)
    with pytest.raises(KeyError):
        promtext.value(fams, "pod_gpu_memory_usage", pid=10)
    assert promtext.value(fams, "amd_gpu_process_vram_bytes", pid=10, gpu=1, pod="") == 300.0


def test_process_exit_removes_series_next_tick(mock_engine):
    e = mock_engine(1, http=False)
    e.mock_set_processes(0, [dict(pid=77, vram_bytes=1.0)])
    e.set_pid_cgroup(77, CG)
    t = ticks(e, 2)
    assert 'pid="77"' in e.snapshot_text()
    e.mock_set_processes(0, [])
    e.tick(t)
    assert 'pid="77"' not in e.snapshot_text()


def test_xgmi_rates_exact(mock_engine):
    e = mock_engine(1, http=False)
    e.mock_set_value(0, "xgmi_read_rate_kbps", 5000.0)
    e.mock_set_value(0, "xgmi_write_rate_kbps", 2000.0)
    ticks(e, 3)
    fams = parse(e)
    rd = promtext.value(fams, "amd_gpu_xgmi_read_bytes_per_second", gpu=0)
    wr = promtext.value(fams, "amd_gpu_xgmi_write_bytes_per_second", gpu=0)
    assert rd == pytest.approx(7 * 5000 * 1024, rel=1e-9)
    assert wr == pytest.approx(7 * 2000 * 1024, rel=1e-9)
    links = [s for s in fams["amd_gpu_xgmi_read_bytes_total"].samples]
    assert len(links) == 7 and all(s[1]["peer_bdf"] for s in links)


def test_counter_reset_and_wrap(mock_engine):
    e = mock_engine(1, http=False)
    e.mock_set_value(0, "xgmi_read_rate_kbps", 1000.0)
    t = ticks(e, 3)
    e.mock_set_fault(0, "counter_reset")
    e.tick(t)
    t += S // 10
    rd = promtext.value(parse(e), "amd_gpu_xgmi_read_bytes_per_second", gpu=0)
    assert rd >= 0  # a reset never produces a negative or huge rate
    assert rd == pytest.approx(7 * 1000 * 1024, rel=1e-6)  # previous rate carried
    e.mock_set_fault(0, "wrap")
    e.tick(t)
    t += S // 10
    e.tick(t)
    rd = promtext.value(parse(e), "amd_gpu_xgmi_read_bytes_per_second", gpu=0)
    assert rd == pytest.approx(7 * 1000 * 1024, rel=1e-6)


def test_energy_counter_monotonic(mock_engine):
    e = mock_engine(1, http=False)
    e.mock_set_value(0, "power_w", 500.0)
    t = ticks(e, 2)
    e1 = promtext.value(parse(e), "amd_gpu_energy_joules_total", gpu=0)
    e.tick(t + S)
    e2 = promtext.value(parse(e), "amd_gpu_energy_joules_total", gpu=0)
    assert e2 - e1 == pytest.approx(500.0 * 1.1, rel=1e-3)


def test_fault_isolation(mock_engine):
    """One failing GPU exports up=0; the others keep reporting (reference: log.Fatalf,
    main.go:119-137)."""
    e = mock_engine(3, http=False)
    t = ticks(e, 2)
    e.mock_set_fault(1, "error")
    t = ticks(e, 2, t)
    fams = parse(e)
    assert promtext.value(fams, "amd_gpu_up", gpu=1) == 0
    assert promtext.value(fams, "amd_gpu_up", gpu=0) == 1
    assert promtext.value(fams, "amd_gpu_up", gpu=2) == 1
    with pytest.raises(KeyError):
        promtext.value(fams, "amd_gpu_power_watts", gpu=1)
    assert promtext.value(fams, "gpuexp_device_errors_total", gpu=1) == 2
    e.mock_set_fault(1, "none")
    ticks(e, 2, t)
    assert promtext.value(parse(e), "amd_gpu_power_watts", gpu=1) > 0


def test_throttle_residency_percent(mock_engine):
    e = mock_engine(1, http=False)
    e.mock_set_value(0, "ppt_residency_percent", 25.0)
    ticks(e, 3, dt=S)
    v = promtext.value(parse(e), "amd_gpu_throttle_residency_percent", gpu=0, reason="ppt")
    assert v == pytest.approx(25.0, abs=0.2)


def test_device_owner_explicit_and_inferred(mock_engine):
    e = mock_engine(2, http=False)
    e.set_pods([dict(uid=UID, namespace="ml", name="trainer-0", containers={CID: "main"})])
    e.set_device_owners({"0000:20:00.0": dict(namespace="infer", pod="server-1", container="srv")})
    e.mock_set_processes(0, [dict(pid=5, vram_bytes=1.0)])
    e.set_pid_cgroup(5, CG)
    ticks(e, 2)
    fams = parse(e)
    up = {s[1]["gpu"]: s[1] for s in fams["amd_gpu_up"].samples}
    assert (up["0"]["namespace"], up["0"]["pod"], up["0"]["container"]) == ("ml", "trainer-0", "main")
    assert (up["1"]["namespace"], up["1"]["pod"]) == ("infer", "server-1")
    assert promtext.value(fams, "amd_pod_gpus", namespace="infer", pod="server-1") == 1
    # owner change relabels: the old series vanish
    e.set_device_owners({})
    e.mock_set_processes(0, [])
    ticks(e, 2, t0=10 * S)
    up = {s[1]["gpu"]: s[1] for s in parse(e)["amd_gpu_up"].samples}
    assert up["1"]["pod"] == "" and up["0"]["pod"] == ""


def test_inferred_owner_follows_control_plane_changes(mock_engine):
    """The single-pod owner inference is reused while the GPU's processes and the control plane
    stay the same: a pod renamed in the pod list, or a PID's cgroup overridden into another
    pod, relabels the GPU at the next tick."""
    e = mock_engine(1, http=False)
    uid2 = "22345678-1234-1234-1234-123456789abc"
    cg2 = CG.replace(UID.replace("-", "_"), uid2.replace("-", "_"))
    e.set_pods([dict(uid=UID, namespace="ml", name="trainer-0", containers={CID: "main"}),
                dict(uid=uid2, namespace="ml", name="other-0", containers={})])
    e.mock_set_processes(0, [dict(pid=5, vram_bytes=1.0)])
    e.set_pid_cgroup(5, CG)
    t = ticks(e, 3)
    owner = lambda: parse(e)["amd_gpu_up"].samples[0][1]["pod"]
    assert owner() == "trainer-0"
    e.set_pods([dict(uid=UID, namespace="ml", name="trainer-1", containers={CID: "main"}),
                dict(uid=uid2, namespace="ml", name="other-0", containers={})])
    t = ticks(e, 2, t)
    assert owner() == "trainer-1"
    e.set_pid_cgroup(5, cg2)
    ticks(e, 2, t)
    assert owner() == "other-0"


def test_shared_gpu_has_no_owner(mock_engine):
    e = mock_engine(1, http=False)
    uid2 = "22345678-1234-1234-1234-123456789abc"
    cg2 = CG.replace(UID.replace("-", "_"), uid2.replace("-", "_"))
    e.mock_set_processes(0, [dict(pid=5, vram_bytes=1.0), dict(pid=6, vram_bytes=2.0)])
    e.set_pid_cgroup(5, CG)
    e.set_pid_cgroup(6, cg2)
    e.set_pods([dict(uid=UID, namespace="a", name="pod-a", containers={}),
                dict(uid=uid2, namespace="b", name="pod-b", containers={})])
    ticks(e, 2)
    fams = parse(e)
    assert fams["amd_gpu_up"].samples[0][1]["pod"] == ""
    assert promtext.value(fams, "amd_pod_gpu_vram_bytes", pod="pod-b") == 2.0
    # one named pod + one not yet named: ownership is unknown, not the named pod's
    e.set_pods([dict(uid=UID, namespace="a", name="pod-a", containers={})])
    ticks(e, 2, t0=10 * S)
    assert parse(e)["amd_gpu_up"].samples[0][1]["pod"] == ""


def test_self_metrics(mock_engine):
    e = mock_engine(1, http=False)
    ticks(e, 5)
    fams = parse(e)
    assert promtext.value(fams, "gpuexp_ticks_total") == 4  # rendered before this tick's count
    assert fams["gpuexp_sample_stage_duration_seconds"].type == "histogram"
    stages = {s[1]["stage"] for s in fams["gpuexp_sample_stage_duration_seconds"].samples}
    assert {"devices", "processes", "render", "series"} <= stages
    st = e.stats()
    assert st["ticks"] == 5 and st["series"] > 60 and st["render_bytes"] > 1000


def test_sampler_thread_runs(native):
    import time
    c = native.EngineConfig()
    c.backend = "mock"
    c.interval_s = 0.01
    c.serve_http = False
    e = native.Engine(c)
    e.start()
    time.sleep(0.3)
    e.stop()
    st = e.stats()
    assert 15 <= st["ticks"] <= 40


def test_full_profile_adds_reliability_families(mock_engine):
    """`full` = the 64-series standard load + ECC / PCIe AER / NAK / recovery / xGMI link
    + per-XCD clocks, per-XCD sentinel dispatch latency and HBM latency (chip + 8 XCDs)
    + the 6 KFD SMI event counters + retired HBM pages by state + GTT used/total + board
    identity and firmware versions + MFMA util + per-XCD MFMA busy + MFMA FLOP/s by type."""
    e = mock_engine(2, http=False, enable_sentinel=True, enable_counters=True, series_profile="full")
    e.mock_set_value(1, "ecc_ue", 3)
    e.mock_set_value(1, "aer_cor", 7)
    ticks(e, 3)
    fams = parse(e)
    # + board (1), firmware (4 in mock), MFMA util (1), per-XCD MFMA busy (8), sentinel pending (1),
    # MFMA FLOP/s for bf16 and fp8 (2), dispatch stall (1), occupancy limiters lds/wave_slots/vgpr/sgpr (4)
    assert dict(device_series_per_gpu(fams)) == {"0": 134, "1": 134}
    lim = {s[1]["resource"]: s[2] for s in fams["amd_gpu_occupancy_limiter_percent"].samples if s[1]["gpu"] == "0"}
    assert lim == {"lds": 80.0, "wave_slots": 10.0, "vgpr": 0.0, "sgpr": 0.0}, lim
    assert promtext.value(fams, "amd_gpu_dispatch_stall_percent", gpu=0) > 0
    flops = {s[1]["dtype"]: s[2] for s in fams["amd_gpu_mfma_flops_per_second"].samples if s[1]["gpu"] == "0"}
    busy = fams["amd_gpu_mfma_busy_percent"].samples[0][2]
    assert flops == {"bf16": pytest.approx(2.5e15 * busy / 100), "fp8": 0.0}, flops
    lat = {s[1]["xcc"]: s[2] for s in fams["amd_gpu_sentinel_xcc_dispatch_latency_seconds"].samples
           if s[1]["gpu"] == "0"}
    assert sorted(lat) == [str(x) for x in range(8)] and min(lat.values()) == lat["0"]
    assert {s[2] for s in fams["amd_gpu_xcc_clock_hz"].samples} == {2.1e9}
    ue = {s[1]["gpu"]: s[2] for s in fams["amd_gpu_ecc_errors_total"].samples
          if s[1]["type"] == "uncorrectable"}
    assert ue == {"0": 0, "1": 3}
    assert {s[1]["severity"] for s in fams["amd_gpu_pcie_aer_errors_total"].samples} == {
        "correctable", "nonfatal", "fatal"}
    assert {s[1]["direction"] for s in fams["amd_gpu_pcie_nak_total"].samples} == {"sent", "received"}
    assert fams["amd_gpu_ecc_errors_total"].type == "counter"


def test_chrome_trace_of_sampler_stages(mock_engine, tmp_path):
    """--trace writes a Chrome-trace (catapult JSON array) of every sampler stage, one
    complete ("X") event per stage per tick, bounded by trace_max_events."""
    import json
    path = tmp_path / "trace.json"
    e = mock_engine(2, http=False, trace_path=str(path), trace_max_events=1000)
    ticks(e, 5)
    e.stop()
    events = [ev for ev in json.loads(path.read_text()) if ev]
    stages = collections.Counter(ev["name"] for ev in events)
    assert {"devices", "processes", "series", "render", "publish"} <= set(stages), stages
    assert len(set(stages.values())) == 1 and stages["render"] == 5  # every stage, every tick
    assert all(ev["ph"] == "X" and ev["dur"] >= 0 for ev in events)
    ts = [ev["ts"] for ev in events]
    assert ts == sorted(ts)
    # bounded: a long-running exporter cannot fill the disk
    path2 = tmp_path / "small.json"
    e2 = mock_engine(1, http=False, trace_path=str(path2), trace_max_events=7)
    ticks(e2, 10)
    e2.stop()
    assert len([ev for ev in json.loads(path2.read_text()) if ev]) == 7


def test_gfx_activity_split_over_processes_and_pods(mock_engine):
    """Shared GPU: the GPU's gfx activity is split by the processes' occupied CUs (KFD has
    no per-process engine time for compute); a sole process gets all of it; pods sum their
    processes' shares over GPUs, so a pod on shared GPUs still gets a utilisation series."""
    e = mock_engine(2, http=False)
    uid2 = "22345678-1234-1234-1234-123456789abc"
    cg2 = CG.replace(UID.replace("-", "_"), uid2.replace("-", "_"))
    for d in (0, 1):
        e.mock_set_value(d, "gfx_activity", 80.0)
    # GPU 0 shared 3:1 by two pods; GPU 1 used only by pod 2's second process
    e.mock_set_processes(0, [dict(pid=5, vram_bytes=1.0, cu_occupancy=96), dict(pid=6, vram_bytes=2.0, cu_occupancy=32)])
    e.mock_set_processes(1, [dict(pid=7, vram_bytes=3.0, cu_occupancy=0)])
    e.set_pid_cgroup(5, CG)
    e.set_pid_cgroup(6, cg2)
    e.set_pid_cgroup(7, cg2)
    e.set_pods([dict(uid=UID, namespace="a", name="pod-1", containers={}),
                dict(uid=uid2, namespace="b", name="pod-2", containers={})])
    ticks(e, 2)
    fams = parse(e)
    share = {s[1]["pid"]: s[2] for s in promtext.samples(fams, "amd_gpu_process_gfx_activity_percent")}
    assert share == {"5": 60.0, "6": 20.0, "7": 80.0}
    pod = {s[1]["pod"]: s[2] for s in promtext.samples(fams, "amd_pod_gfx_activity_share_percent")}
    assert pod == {"pod-1": 60.0, "pod-2": 100.0}  # 20% of GPU 0 + 80% of GPU 1
    # nothing resident at the CU sample: an even split, never a division by zero
    e.mock_set_processes(0, [dict(pid=5, cu_occupancy=0), dict(pid=6, cu_occupancy=0)])
    ticks(e, 1, t0=10 * S)
    share = {s[1]["pid"]: s[2] for s in promtext.samples(parse(e), "amd_gpu_process_gfx_activity_percent")}
    assert share["5"] == share["6"] == 40.0


def test_pod_energy_from_hardware_counters(native, mock_engine):
    """amd_pod_gpu_energy_joules_total: an owned GPU's energy counter goes to its pod; a
    shared GPU's is split by the processes' CU-occupancy shares; totals persist while the
    control plane knows the pod."""
    uids = {p: f"00000000-0000-4000-8000-00000000000{i}" for i, p in enumerate("abc", 1)}
    cids = {p: p * 64 for p in "abc"}
    e = mock_engine(2, series_profile="standard")
    e.set_pods([{"uid": uids[p], "namespace": "ns", "name": f"pod-{p}", "containers": {cids[p]: "w"}} for p in "abc"])
    for pid, p in ((100, "a"), (200, "b"), (300, "c")):
        e.set_pid_cgroup(pid, kubepods_cgroup(uids[p], cids[p]))
    e.set_device_owners({"0000:10:00.0": {"namespace": "ns", "pod": "pod-a", "container": "w"}})
    e.mock_set_value(0, "power_w", 500)
    e.mock_set_value(1, "power_w", 800)
    e.mock_set_processes(0, [{"pid": 100, "vram_bytes": 1 << 30, "cu_occupancy": 200, "name": "a"}])
    e.mock_set_processes(1, [{"pid": 200, "vram_bytes": 1 << 30, "cu_occupancy": 48, "name": "b"},
                             {"pid": 300, "vram_bytes": 1 << 30, "cu_occupancy": 16, "name": "c"}])
    for t in range(1, 5):  # 3 one-second intervals
        e.tick(t * 1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    en = {s[1]["pod"]: s[2] for s in promtext.samples(fams, "amd_pod_gpu_energy_joules_total")}
    assert en["pod-a"] == pytest.approx(3 * 500, rel=0.01)
    assert en["pod-b"] == pytest.approx(3 * 800 * 0.75, rel=0.01)
    assert en["pod-c"] == pytest.approx(3 * 800 * 0.25, rel=0.01)
    # pod-c's process exits: its total stays; the pod leaves the control plane: it goes
    e.mock_set_processes(1, [{"pid": 200, "vram_bytes": 1 << 30, "cu_occupancy": 48, "name": "b"}])
    e.tick(5 * 1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    en2 = {s[1]["pod"]: s[2] for s in promtext.samples(fams, "amd_pod_gpu_energy_joules_total")}
    assert en2["pod-c"] == pytest.approx(en["pod-c"]) and en2["pod-b"] == pytest.approx(en["pod-b"] + 800, rel=0.01)
    e.set_pods([{"uid": uids[p], "namespace": "ns", "name": f"pod-{p}", "containers": {cids[p]: "w"}} for p in "ab"])
    e.tick(6 * 1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    assert "pod-c" not in {s[1]["pod"] for s in promtext.samples(fams, "amd_pod_gpu_energy_joules_total")}


def test_state_file_carries_pod_totals_across_restarts(native, mock_engine, tmp_path):
    """Checkpoint/resume of the exporter's own accumulations: per-pod energy and KFD event
    counts, and per-GPU event counts, continue from the state file after a restart (kept
    until the control plane has delivered its pod list, then GC'd as usual)."""
    state = str(tmp_path / "state")
    uid, cid = "00000000-0000-4000-8000-0000000000aa", "ab" * 32
    pods = [{"uid": uid, "namespace": "ns", "name": "trainer", "containers": {cid: "w"}}]

    def engine():
        e = mock_engine(1, series_profile="full", state_file=state)
        e.mock_set_value(0, "power_w", 400)
        e.mock_set_processes(0, [{"pid": 100, "vram_bytes": 1 << 30, "cu_occupancy": 10, "name": "t"}])
        e.set_pid_cgroup(100, kubepods_cgroup(uid, cid))
        return e

    def totals(e):
        f = promtext.parse(e.snapshot_text())
        en = {s[1]["pod"]: s[2] for s in promtext.samples(f, "amd_pod_gpu_energy_joules_total")}
        pev = {(s[1]["pod"], s[1]["event"]): s[2] for s in promtext.samples(f, "amd_pod_gpu_kfd_events_total")}
        dev = {s[1]["event"]: s[2] for s in promtext.samples(f, "amd_gpu_kfd_events_total")}
        busy = {s[1]["pod"]: s[2] for s in promtext.samples(f, "amd_pod_gpu_busy_seconds_total")}
        return en, pev, dev, busy

    a = engine()
    a.set_pods(pods)
    a.inject_kfd_events(0, b"1 64:t\n2 0:1\n")
    for t in range(1, 5):
        a.tick(t * 1_000_000_000)
    en1, pev1, dev1, busy1 = totals(a)
    assert en1["trainer"] == pytest.approx(3 * 400, rel=0.01) and pev1[("trainer", "vm_fault")] == 1
    assert 0 < busy1["trainer"] <= 3.0  # the sole process of a shared GPU: all its busy time
    a.stop()  # final save
    assert open(state).read().startswith("gpuexp-state 1\n")

    b = engine()
    assert "restored" in b.source_status()
    b.tick(10_000_000_000)  # no pod list yet: restored totals are kept, not GC'd
    en2, pev2, dev2, busy2 = totals(b)
    assert en2 == en1 and pev2 == pev1 and dev2["vm_fault"] == 1 and dev2["thermal_throttle"] == 1
    assert busy2 == busy1
    b.set_pods(pods)
    for t in range(11, 14):
        b.tick(t * 1_000_000_000)
    en3, _, _, busy3 = totals(b)
    assert busy3["trainer"] > busy1["trainer"]
    assert en3["trainer"] == pytest.approx(en1["trainer"] + 3 * 400, rel=0.01)  # continues, no reset
    b.set_pods([])
    b.tick(14_000_000_000)
    assert not totals(b)[0]  # the pod is gone: its total goes with it
    b.stop()


def test_state_file_with_unknown_format_is_ignored(native, mock_engine, tmp_path):
    state = tmp_path / "state"
    state.write_text("something else\npod_energy\tns\tp\t1e9\n")
    e = mock_engine(1, series_profile="full", state_file=str(state))
    assert "ignored" in e.source_status()
    e.tick(1_000_000_000)
    assert not promtext.samples(promtext.parse(e.snapshot_text()), "amd_pod_gpu_energy_joules_total")


def test_pod_xgmi_byte_counters(native, mock_engine, tmp_path):
    """amd_pod_xgmi_{read,write}_bytes_total: per-tick xGMI link-accumulator deltas of the
    pod's GPUs (an owned GPU's whole, a shared GPU's by CU-occupancy share), kept while the
    control plane knows the pod, moved with an ownership change, not dropped by an
    incomplete refresh, and carried across an exporter restart by the state file."""
    state = str(tmp_path / "state")
    uids = {p: f"00000000-0000-4000-8000-00000000001{i}" for i, p in enumerate("abc", 1)}
    cids = {p: p * 64 for p in "abc"}
    K = 7 * 1024  # 7 links per mock GPU, kB -> B
    pods = [{"uid": uids[p], "namespace": "ns", "name": f"pod-{p}", "containers": {cids[p]: "w"}} for p in "abc"]

    def engine():
        e = mock_engine(2, series_profile="standard", state_file=state)
        for pid, p in ((100, "a"), (200, "b"), (300, "c")):
            e.set_pid_cgroup(pid, kubepods_cgroup(uids[p], cids[p]))
        e.mock_set_value(0, "xgmi_read_rate_kbps", 1000)
        e.mock_set_value(0, "xgmi_write_rate_kbps", 2000)
        e.mock_set_value(1, "xgmi_read_rate_kbps", 4000)
        e.mock_set_value(1, "xgmi_write_rate_kbps", 0)
        e.mock_set_processes(0, [{"pid": 100, "vram_bytes": 1 << 30, "cu_occupancy": 200, "name": "a"}])
        e.mock_set_processes(1, [{"pid": 200, "vram_bytes": 1 << 30, "cu_occupancy": 48, "name": "b"},
                                 {"pid": 300, "vram_bytes": 1 << 30, "cu_occupancy": 16, "name": "c"}])
        return e

    def totals(e):
        f = promtext.parse(e.snapshot_text())
        rd = {s[1]["pod"]: s[2] for s in promtext.samples(f, "amd_pod_xgmi_read_bytes_total")}
        wr = {s[1]["pod"]: s[2] for s in promtext.samples(f, "amd_pod_xgmi_write_bytes_total")}
        return rd, wr

    e = engine()
    e.set_pods(pods)
    e.set_device_owners({"0000:10:00.0": {"namespace": "ns", "pod": "pod-a", "container": "w"}})
    for t in range(1, 5):  # 3 one-second intervals
        e.tick(t * S)
    rd, wr = totals(e)
    assert rd["pod-a"] == pytest.approx(3 * 1000 * K, rel=1e-3) and wr["pod-a"] == pytest.approx(3 * 2000 * K, rel=1e-3)
    assert rd["pod-b"] == pytest.approx(3 * 4000 * K * 0.75, rel=1e-3)
    assert rd["pod-c"] == pytest.approx(3 * 4000 * K * 0.25, rel=1e-3) and wr["pod-c"] == 0
    # GPU 0 changes hands: its bytes from now on are pod-b's; pod-a keeps what it had
    e.set_device_owners({"0000:10:00.0": {"namespace": "ns", "pod": "pod-b", "container": "w"}})
    e.tick(5 * S)
    rd2, wr2 = totals(e)
    assert rd2["pod-a"] == pytest.approx(rd["pod-a"])
    assert rd2["pod-b"] == pytest.approx(rd["pod-b"] + 1000 * K + 4000 * K * 0.75, rel=1e-3)
    # a refresh in which a source failed (pod-c missing from it) drops nothing...
    e.set_pods(pods[:2], False)
    e.tick(6 * S)
    assert "pod-c" in totals(e)[0]
    # ...a complete one without pod-c does
    e.set_pods(pods[:2])
    e.tick(7 * S)
    rd3, _ = totals(e)
    assert "pod-c" not in rd3
    e.stop()  # final save
    assert "pod_xgmi\tns\tpod-a\t" in open(state).read()

    b = engine()
    b.tick(10 * S)  # no pod list yet: restored totals exported as they were
    assert totals(b)[0]["pod-a"] == pytest.approx(rd3["pod-a"])
    b.set_pods(pods[1:2], False)  # an incomplete first refresh without pod-a (apiserver down)...
    b.tick(11 * S)
    assert totals(b)[0]["pod-a"] == pytest.approx(rd3["pod-a"])  # ...keeps pod-a's restored total
    b.set_pods(pods[1:2])  # a complete one without it drops it
    b.tick(12 * S)
    assert "pod-a" not in totals(b)[0]
    b.stop()


def test_xcc_mfma_busy_series(mock_engine):
    """amd_gpu_xcc_mfma_busy_percent: one series per XCD of the GPU, full profile only,
    from the same counter window as the chip value."""
    e = mock_engine(1, http=False, enable_counters=True, series_profile="full")
    e.mock_set_value(0, "mfma_busy_pct", 30.0)
    e.mock_set_value(0, "xcc_mfma_busy_pct", 30.0)
    ticks(e, 2)
    fams = parse(e)
    xs = {s[1]["xcc"]: s[2] for s in fams["amd_gpu_xcc_mfma_busy_percent"].samples if s[1]["gpu"] == "0"}
    assert sorted(xs) == [str(x) for x in range(8)] and set(xs.values()) == {30.0}
    assert promtext.value(fams, "amd_gpu_mfma_busy_percent", gpu=0) == 30.0
    std = mock_engine(1, http=False, enable_counters=True)
    ticks(std, 2)
    assert "amd_gpu_xcc_mfma_busy_percent" not in parse(std)


def test_sentinel_pending_seconds(mock_engine):
    """amd_gpu_sentinel_pending_seconds (full profile): 0 while runs complete, the scripted
    wait while one is outstanding."""
    e = mock_engine(1, http=False, enable_sentinel=True, series_profile="full")
    ticks(e, 2)
    assert promtext.value(parse(e), "amd_gpu_sentinel_pending_seconds", gpu=0) == 0.0
    e.mock_set_value(0, "sentinel_pending_s", 75.0)
    ticks(e, 1, t0=10 * S)
    assert promtext.value(parse(e), "amd_gpu_sentinel_pending_seconds", gpu=0) == 75.0


def test_pod_gpu_seconds(native, mock_engine):
    """amd_pod_gpu_allocated_seconds_total / amd_pod_gpu_busy_seconds_total: GPU-seconds a pod
    held its GPUs, and how many of them they were busy (the mean per-XCD busy of each tick,
    times the tick)."""
    uid, cid = "00000000-0000-4000-8000-0000000000c3", "c3" * 32
    e = mock_engine(2)
    e.set_pods([{"uid": uid, "namespace": "ml", "name": "holder", "containers": {cid: "w"}}])
    e.set_device_owners({"0000:10:00.0": {"namespace": "ml", "pod": "holder", "container": "w"},
                         "0000:20:00.0": {"namespace": "ml", "pod": "holder", "container": "w"}})
    busy = 0.0
    for t in range(1, 6):  # 4 one-second ticks after the first
        e.tick(t * 1_000_000_000)
        fams = promtext.parse(e.snapshot_text())
        if t > 1:
            for g in ("0", "1"):
                xs = [s[2] for s in promtext.samples(fams, "amd_gpu_xcc_busy_percent") if s[1]["gpu"] == g]
                busy += sum(xs) / len(xs) / 100.0
    alloc = promtext.value(fams, "amd_pod_gpu_allocated_seconds_total", pod="holder")
    got = promtext.value(fams, "amd_pod_gpu_busy_seconds_total", pod="holder")
    assert alloc == pytest.approx(8.0)  # 2 GPUs x 4 s
    assert 0 < got <= alloc and got == pytest.approx(busy, rel=1e-6)


def test_pod_hbm_bandwidth_is_the_sum_of_its_gpus(native, mock_engine):
    """amd_pod_gpu_hbm_bandwidth_bytes_per_second: the HBM bandwidth of the GPUs a pod owns,
    summed (the same PMFW-derived value as amd_gpu_hbm_bandwidth_bytes_per_second)."""
    uid, cid = "00000000-0000-4000-8000-0000000000c2", "c2" * 32
    e = mock_engine(3)
    e.set_pods([{"uid": uid, "namespace": "ml", "name": "reader", "containers": {cid: "w"}}])
    e.set_device_owners({"0000:10:00.0": {"namespace": "ml", "pod": "reader", "container": "w"},
                         "0000:20:00.0": {"namespace": "ml", "pod": "reader", "container": "w"}})
    e.tick(S)
    e.tick(2 * S)
    fams = promtext.parse(e.snapshot_text())
    g = [promtext.value(fams, "amd_gpu_hbm_bandwidth_bytes_per_second", gpu=i) for i in range(3)]
    assert g[0] > 0 and g[1] > 0
    pod = promtext.value(fams, "amd_pod_gpu_hbm_bandwidth_bytes_per_second", pod="reader")
    assert abs(pod - (g[0] + g[1])) <= 1e-6 * pod


def test_pod_mfma_busy_is_the_mean_of_its_gpus(native, mock_engine):
    """amd_pod_gpu_mfma_busy_percent: the mean MFMA busy of the GPUs a pod owns (device
    plugin map), from the same per-tick counter window as amd_gpu_mfma_busy_percent."""
    uid, cid = "00000000-0000-4000-8000-0000000000c1", "c1" * 32
    e = mock_engine(3, enable_counters=True)
    e.set_pods([{"uid": uid, "namespace": "ml", "name": "trainer", "containers": {cid: "w"}}])
    e.set_device_owners({"0000:10:00.0": {"namespace": "ml", "pod": "trainer", "container": "w"},
                         "0000:20:00.0": {"namespace": "ml", "pod": "trainer", "container": "w"}})
    e.mock_set_value(0, "mfma_busy_pct", 80.0)
    e.mock_set_value(1, "mfma_busy_pct", 40.0)
    e.mock_set_value(2, "mfma_busy_pct", 5.0)  # not the pod's
    e.tick(S)
    e.tick(2 * S)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "amd_gpu_mfma_busy_percent", gpu=0) == 80.0
    assert promtext.value(fams, "amd_pod_gpu_mfma_busy_percent", pod="trainer") == 60.0


def test_mfma_flops_by_type_per_gpu_and_pod(native, mock_engine):
    """amd_gpu_mfma_flops_per_second{dtype} (SQ_INSTS_VALU_MFMA_MOPS_<type> x 512, full
    profile, device-scope counters only) and amd_pod_gpu_mfma_flops_per_second: the sum over
    the GPUs a pod owns, per operand type."""
    uid, cid = "00000000-0000-4000-8000-0000000000c2", "c2" * 32
    e = mock_engine(3, enable_counters=True, series_profile="full")
    e.set_pods([{"uid": uid, "namespace": "ml", "name": "trainer", "containers": {cid: "w"}}])
    e.set_device_owners({"0000:10:00.0": {"namespace": "ml", "pod": "trainer", "container": "w"},
                         "0000:20:00.0": {"namespace": "ml", "pod": "trainer", "container": "w"}})
    e.mock_set_value(0, "mfma_bf16_flops", 1.2e15)
    e.mock_set_value(1, "mfma_bf16_flops", 0.8e15)
    e.mock_set_value(1, "mfma_fp8_flops", 2.0e15)
    e.mock_set_value(2, "mfma_bf16_flops", 9e14)  # not the pod's
    e.tick(S)
    e.tick(2 * S)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "amd_gpu_mfma_flops_per_second", gpu=1, dtype="fp8") == 2.0e15
    assert promtext.value(fams, "amd_pod_gpu_mfma_flops_per_second", pod="trainer", dtype="bf16") == 2.0e15
    assert promtext.value(fams, "amd_pod_gpu_mfma_flops_per_second", pod="trainer", dtype="fp8") == 2.0e15
    # standard profile: the 64-series load without the per-type FLOP families
    e2 = mock_engine(1, enable_counters=True, series_profile="standard")
    e2.tick(S)
    e2.tick(2 * S)
    assert "amd_gpu_mfma_flops_per_second" not in promtext.parse(e2.snapshot_text())


def test_pod_gpu_seconds_on_a_shared_gpu(native, mock_engine):
    """A GPU no device plugin owns, used by two pods' processes 3:1 by CU occupancy: each pod is
    credited that share of the GPU's time as allocated AND of its busy time, so busy <= allocated
    for both (round 3 credited busy only: busy / allocated was +Inf for such pods)."""
    uids = {p: f"00000000-0000-4000-8000-0000000000d{i}" for i, p in enumerate("ab", 1)}
    cids = {p: p * 64 for p in "ab"}
    e = mock_engine(1)
    e.set_pods([{"uid": uids[p], "namespace": "ns", "name": f"pod-{p}", "containers": {cids[p]: "w"}} for p in "ab"])
    e.set_pid_cgroup(100, kubepods_cgroup(uids["a"], cids["a"]))
    e.set_pid_cgroup(200, kubepods_cgroup(uids["b"], cids["b"]))
    e.mock_set_processes(0, [{"pid": 100, "vram_bytes": 1 << 30, "cu_occupancy": 48, "name": "a"},
                             {"pid": 200, "vram_bytes": 1 << 30, "cu_occupancy": 16, "name": "b"}])
    for t in range(1, 6):  # 4 one-second ticks after the first
        e.tick(t * S)
    fams = promtext.parse(e.snapshot_text())
    alloc = {s[1]["pod"]: s[2] for s in promtext.samples(fams, "amd_pod_gpu_allocated_seconds_total")}
    busy = {s[1]["pod"]: s[2] for s in promtext.samples(fams, "amd_pod_gpu_busy_seconds_total")}
    assert alloc["pod-a"] == pytest.approx(4 * 0.75) and alloc["pod-b"] == pytest.approx(4 * 0.25)
    for p in ("pod-a", "pod-b"):
        assert 0 < busy[p] <= alloc[p], (p, busy, alloc)


def test_pod_totals_expire_under_partial_pod_lists(native, mock_engine):
    """Per-pod totals of a pod that left are dropped at once by a complete pod list; while every
    refresh is partial (a metadata source keeps failing) they are kept, but only for
    pod_totals_ttl, and gpuexp_pod_list_complete says which case applies."""
    import time
    uid, cid = "00000000-0000-4000-8000-0000000000e1", "e1" * 32
    e = mock_engine(1, pod_totals_ttl_s=0.5)
    e.set_pods([{"uid": uid, "namespace": "ns", "name": "gone", "containers": {cid: "w"}}], True)
    e.set_pid_cgroup(100, kubepods_cgroup(uid, cid))
    e.mock_set_processes(0, [{"pid": 100, "vram_bytes": 1 << 30, "cu_occupancy": 48, "name": "a"}])
    e.tick(S)
    e.tick(2 * S)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "gpuexp_pod_list_complete") == 1
    assert promtext.value(fams, "amd_pod_gpu_energy_joules_total", pod="gone") > 0
    e.mock_set_processes(0, [])
    e.set_pods([], False)  # partial refresh without the pod: totals kept...
    e.tick(3 * S)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "gpuexp_pod_list_complete") == 0
    assert promtext.value(fams, "amd_pod_gpu_energy_joules_total", pod="gone") > 0
    time.sleep(0.6)  # ...until no applied list has had the pod for the TTL
    e.set_pods([], False)
    e.tick(4 * S)
    fams = promtext.parse(e.snapshot_text())
    assert not promtext.samples(fams, "amd_pod_gpu_energy_joules_total")
    assert not promtext.samples(fams, "amd_pod_gpu_allocated_seconds_total")
