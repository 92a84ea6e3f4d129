"""KFD SMI events (kfd_events.cc): the message parser, and per-GPU / per-pod counting in the
engine fed through the injection hook (the real source reads /dev/kfd event fds on a GPU
box; tests/test_gpu.py::test_kfd_events_source_opens)."""
import pytest

from kubernetes_gpu_exporter_amd.utils import promtext
from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup

UID = "11111111-2222-4333-8444-555555555555"
CID = "ab" * 32


@pytest.mark.parametrize("line,want", [
    (b"1 1092:python3", ("vm_fault", 0x1092)),          # "<pid hex>:<comm>"
    (b"2 1:3", ("thermal_throttle", -1)),               # "<bitmask>:<counter>", device-wide
    (b"3 5 RAS_FATAL", ("gpu_pre_reset", -1)),
    (b"4 5", ("gpu_post_reset", -1)),
    (b"9 1234567890 -4242 1 2", ("queue_eviction", 4242)),   # "<ns> -<pid dec> <node> <trigger>"
    (b"a 1234567890 -77 1 Y", ("queue_restore", 77)),
    (b"7 99 -12 @7f00(1) R", ("page_fault_start", 12)),
])
def test_parse_kfd_event(native, line, want):
    assert native.parse_kfd_event(line) == want


@pytest.mark.parametrize("line", [b"", b"zz", b"1", b"1 :x", b"0 1", b"c 1", b"9 123 77 1", b"9 123 - 1"])
def test_parse_kfd_event_rejects(native, line):
    assert native.parse_kfd_event(line) is None


def _kfd(fams, gpu, event):
    v = [s[2] for s in promtext.samples(fams, "amd_gpu_kfd_events_total")
         if s[1]["gpu"] == gpu and s[1]["event"] == event]
    assert len(v) == 1, (gpu, event, v)
    return v[0]


def test_engine_counts_kfd_events_per_gpu_and_pod(native, mock_engine):
    e = mock_engine(2, series_profile="full")
    e.set_pods([{"uid": UID, "namespace": "ml", "name": "trainer-0", "containers": {CID: "main"}}])
    e.set_pid_cgroup(4242, kubepods_cgroup(UID, CID))
    e.tick(1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    # every subscribed event exists from the start, at 0, on every GPU
    assert len(promtext.samples(fams, "amd_gpu_kfd_events_total")) == 2 * 6
    assert _kfd(fams, "1", "vm_fault") == 0
    assert [s for s in promtext.samples(fams, "gpuexp_source_up") if s[1]["source"] == "kfd_events"][0][2] == 1

    # GPU 1: a VM fault and a queue eviction of pid 4242 (the pod's), one of an unknown pid;
    # GPU 0: a thermal-throttle message split over two reads, and one malformed line
    e.inject_kfd_events(1, b"1 1092:python3\n9 100 -4242 0 2\n1 f423f:other\n")
    e.inject_kfd_events(0, b"2 0:")
    e.inject_kfd_events(0, b"1\nnot an event\n")
    e.tick(1_100_000_000)
    fams = promtext.parse(e.snapshot_text())
    assert _kfd(fams, "1", "vm_fault") == 2 and _kfd(fams, "1", "queue_eviction") == 1
    assert _kfd(fams, "0", "thermal_throttle") == 1 and _kfd(fams, "0", "vm_fault") == 0
    pod = {(s[1]["namespace"], s[1]["pod"], s[1]["event"]): s[2]
           for s in promtext.samples(fams, "amd_pod_gpu_kfd_events_total")}
    assert pod == {("ml", "trainer-0", "vm_fault"): 1, ("ml", "trainer-0", "queue_eviction"): 1}

    # counts survive a change of the GPU's owner labels, and the pod's vanish with the pod
    e.set_device_owners({"0000:20:00.0": {"namespace": "ml", "pod": "trainer-0", "container": "main"}})
    e.set_pods([])
    e.tick(1_200_000_000)
    fams = promtext.parse(e.snapshot_text())
    s1 = [s for s in promtext.samples(fams, "amd_gpu_kfd_events_total") if s[1]["gpu"] == "1"]
    assert {s[1]["pod"] for s in s1} == {"trainer-0"}
    assert _kfd(fams, "1", "vm_fault") == 2
    assert not promtext.samples(fams, "amd_pod_gpu_kfd_events_total")


def test_kfd_events_full_profile_only(native, mock_engine):
    e = mock_engine(1, series_profile="standard")
    e.inject_kfd_events(0, b"1 1092:python3\n")
    e.tick(1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    assert not promtext.samples(fams, "amd_gpu_kfd_events_total")
    off = mock_engine(1, series_profile="full", enable_kfd_events=False)
    off.tick(1_000_000_000)
    assert not promtext.samples(promtext.parse(off.snapshot_text()), "amd_gpu_kfd_events_total")



def test_pod_kfd_event_totals_expire_under_partial_pod_lists(native, mock_engine):
    """Per-pod KFD event counts follow the same TTL as the other per-pod totals while every pod
    refresh is partial: kept for pod_totals_ttl_s after the last list that had the pod, then
    dropped (not kept for ever once the pod's energy totals expired first)."""
    import time
    e = mock_engine(1, series_profile="full", pod_totals_ttl_s=0.5)
    e.set_pods([{"uid": UID, "namespace": "ml", "name": "gone", "containers": {CID: "main"}}], True)
    e.set_pid_cgroup(4242, kubepods_cgroup(UID, CID))
    e.mock_set_processes(0, [{"pid": 4242, "vram_bytes": 1 << 30, "cu_occupancy": 8, "name": "a"}])
    e.tick(1_000_000_000)
    e.inject_kfd_events(0, b"1 1092:python3\n")
    e.tick(1_100_000_000)
    pod = lambda f: {(s[1]["pod"], s[1]["event"]): s[2] for s in promtext.samples(f, "amd_pod_gpu_kfd_events_total")}
    assert pod(promtext.parse(e.snapshot_text())) == {("gone", "vm_fault"): 1}
    e.mock_set_processes(0, [])
    e.set_pods([], False)  # partial refreshes without the pod: kept ...
    e.tick(1_200_000_000)
    assert pod(promtext.parse(e.snapshot_text())) == {("gone", "vm_fault"): 1}
    time.sleep(0.6)  # ... until no applied list has had the pod for the TTL
    for t in (1_300_000_000, 1_400_000_000, 1_500_000_000):
        e.set_pods([], False)
        e.tick(t)
    fams = promtext.parse(e.snapshot_text())
    assert not promtext.samples(fams, "amd_pod_gpu_energy_joules_total")
    assert pod(fams) == {}


def test_drain_polls_every_gpu_fd_and_reads_only_the_ready_ones(native):
    """KfdEventSource.drain: one poll over all GPUs' event fds, then reads of the readable ones
    (pipes stand in for KFD's SMI event fds): events of two GPUs among four, a trailing partial
    line kept back, and a second drain with every fd quiet."""
    import os
    pipes = [os.pipe() for _ in range(4)]
    for r, _ in pipes:
        os.set_blocking(r, False)
    os.write(pipes[1][1], b"1 1092:python3\n")              # GPU 1: a VM fault of pid 0x1092
    os.write(pipes[3][1], b"9 100 -4242 0 2\n2 0:")         # GPU 3: an eviction of 4242 + half a line
    # two drains: the second finds every fd quiet (the poll returns 0, nothing is read)
    got = native.kfd_events_drain_fds([r for r, _ in pipes], 2)  # (the source owns and closes the read ends)
    assert sorted(got) == [(1, 1, 0x1092), (3, 9, 4242)], got
    for _, w in pipes:
        os.close(w)
