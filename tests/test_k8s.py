"""Control plane against fake kubelet (PodResources gRPC) and fake apiserver, plus the
full exporter on a fake host root: device -> pod via the device plugin, PID -> pod via
cgroups, pod UID -> namespace/name via a node-scoped pod list."""
import os
import time

import pytest

from kubernetes_gpu_exporter_amd.config import make_config
from kubernetes_gpu_exporter_amd.k8s.controlplane import ControlPlane, Metadata
from kubernetes_gpu_exporter_amd.k8s.fakes import FakeApiserver, FakeKubelet, FakePod
from kubernetes_gpu_exporter_amd.k8s.filesource import FileSource, write_pod_map
from kubernetes_gpu_exporter_amd.k8s.podresources import PodResourcesSource
from kubernetes_gpu_exporter_amd.k8s.sources import ApiserverSource, LogdirSource, strip_container_id
from kubernetes_gpu_exporter_amd.utils import promtext
from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup, mi355x_node

UID_A = "aaaaaaaa-0000-4000-8000-000000000001"
UID_B = "bbbbbbbb-0000-4000-8000-000000000002"
UID_C = "cccccccc-0000-4000-8000-000000000003"
CID_A = "a1" * 32
CID_B = "b2" * 32


def pods():
    return [
        FakePod(UID_A, "research", "llama-train-0", "node-a", {"trainer": CID_A}, {"trainer": ["0000:72:00.0"]}),
        FakePod(UID_B, "serving", "vllm-0", "node-a", {"server": CID_B, "sidecar": "c3" * 32},
                {"server": ["0000:5a:00.0"]}),
        FakePod(UID_C, "other", "elsewhere", "node-b", {"x": "d4" * 32}, {"x": ["0000:23:00.0"]}),
    ]


def test_strip_container_id():
    assert strip_container_id("containerd://abc") == "abc"
    assert strip_container_id("cri-o://abc") == "abc"
    assert strip_container_id("abc") == "abc"  # reference sliced from offset 2 here (main.go:97)
    assert strip_container_id("") == ""


def test_podresources_roundtrip(tmp_path):
    sock = str(tmp_path / "kubelet.sock")
    k = FakeKubelet(sock, pods()).start()
    try:
        md = PodResourcesSource(sock).fetch()
        assert md.owners["0000:72:00.0"] == {"namespace": "research", "pod": "llama-train-0", "container": "trainer"}
        assert md.owners["0000:5a:00.0"]["container"] == "server"
        assert len(md.owners) == 3  # the kubelet only reports its own node; the fake reports all
        k.fail = True
        with pytest.raises(Exception):
            PodResourcesSource(sock).fetch()
    finally:
        k.stop()


def test_podresources_timeout(tmp_path):
    sock = str(tmp_path / "kubelet.sock")
    k = FakeKubelet(sock, pods()).start()
    k.delay = 1.0
    try:
        t0 = time.monotonic()
        with pytest.raises(Exception):
            PodResourcesSource(sock, timeout=0.2).fetch()
        assert time.monotonic() - t0 < 0.9
    finally:
        k.stop()


def test_apiserver_node_scoped(tmp_path):
    api = FakeApiserver(pods(), token="s3cret").start()
    tok = tmp_path / "token"
    tok.write_text("s3cret\n")
    try:
        md = ApiserverSource(api.url, "node-a", str(tok), watch=False).fetch()
        assert set(md.pods) == {UID_A, UID_B}  # node-b pod excluded (reference listed ALL pods)
        assert md.pods[UID_B]["containers"][CID_B] == "server"
        assert md.pods[UID_A]["namespace"] == "research"
        assert "fieldSelector=spec.nodeName%3Dnode-a" in api.requests[-1]
        assert "resourceVersion=0" in api.requests[-1]
        with pytest.raises(Exception):
            ApiserverSource(api.url, "node-a", "", watch=False).fetch()  # no token -> 401
    finally:
        api.stop()


def test_logdir_source(tmp_path):
    d = tmp_path / "var/log/pods"
    (d / f"research_llama-train-0_{UID_A}/trainer").mkdir(parents=True)
    (d / f"kube-system_my_weird_name_{UID_B}/c").mkdir(parents=True)
    (d / "garbage").mkdir()
    md = LogdirSource(str(d)).fetch()
    assert md.pods[UID_A]["name"] == "llama-train-0"
    assert md.pods[UID_B]["name"] == "my_weird_name" and md.pods[UID_B]["namespace"] == "kube-system"
    assert len(md.pods) == 2


def test_file_source_reload(tmp_path):
    p = str(tmp_path / "map.json")
    write_pod_map(p, [{"uid": UID_A, "namespace": "n", "name": "a", "containers": {}}], {123: "/kubepods/x"})
    s = FileSource(p)
    assert s.fetch().pid_cgroups == {123: "/kubepods/x"}
    time.sleep(0.01)
    write_pod_map(p, [{"uid": UID_B, "namespace": "n", "name": "b", "containers": {}}])
    os.utime(p, ns=(time.time_ns() + 10**6, time.time_ns() + 10**6))
    assert list(s.fetch().pods) == [UID_B]


class _Boom:
    name = "boom"

    def fetch(self):
        raise RuntimeError("apiserver 503")


class _Static:
    name = "static"

    def __init__(self, md):
        self.md = md

    def fetch(self):
        return self.md


def test_control_plane_isolates_failures_and_pushes_on_change(mock_engine):
    e = mock_engine(1, http=False)
    md = Metadata(pods={UID_A: {"uid": UID_A, "namespace": "ns", "name": "p", "containers": {}}},
                  pid_cgroups={42: kubepods_cgroup(UID_A, CID_A)})
    cp = ControlPlane([_Boom(), _Static(md)], interval=0.05)
    cp.attach(e)
    cp.refresh_once()
    assert "boom" in cp.errors
    e.mock_set_processes(0, [dict(pid=42, vram_bytes=7.0)])
    e.tick(1_000_000_000)
    assert promtext.value(promtext.parse(e.snapshot_text()), "pod_gpu_memory_usage", pid="42", pod="p") == 7
    # unchanged metadata is not re-pushed
    fp = cp._last_fp
    cp.refresh_once()
    assert cp._last_fp == fp


def test_control_plane_skips_unchanged_cached_sources(tmp_path):
    """A FileSource hands back its cached Metadata until the file changes: the refresh then
    skips the merge and fingerprint (and pushes nothing); a new file is pushed again."""
    p = str(tmp_path / "map.json")
    write_pod_map(p, [{"uid": UID_A, "namespace": "n", "name": "a", "containers": {}}])

    class _Eng:
        def __init__(self):
            self.pushes = 0

        def set_pods(self, pods, complete):
            self.pushes += 1

        def set_device_owners(self, owners):
            pass

        def set_pid_cgroup(self, pid, path):
            pass

        def clear_pid_cgroups(self):
            pass

    eng = _Eng()
    cp = ControlPlane([FileSource(p)], interval=0.05)
    cp.attach(eng)
    first = cp.refresh_once()
    assert eng.pushes == 1 and list(first.pods) == [UID_A]
    assert cp.refresh_once() is first and cp.refreshes == 2 and eng.pushes == 1
    write_pod_map(p, [{"uid": UID_B, "namespace": "n", "name": "b", "containers": {}}])
    os.utime(p, ns=(time.time_ns() + 10**6, time.time_ns() + 10**6))
    assert list(cp.refresh_once().pods) == [UID_B] and eng.pushes == 2


def test_failed_refresh_never_drops_restored_pod_totals(mock_engine, tmp_path):
    """the first refresh runs while the apiserver is down.  Its (partial) pod
    list must not garbage-collect the per-pod totals restored from --state-file; the first
    complete refresh does, for pods that are really gone."""
    state = tmp_path / "state"
    state.write_text("gpuexp-state 1\npod_energy\tns\tgone\t123\npod_energy\tns\tp\t7\n"
                     "pod_xgmi\tns\tgone\t1000\t2000\n")
    e = mock_engine(1, http=False, series_profile="full", state_file=str(state))
    md = Metadata(pods={UID_A: {"uid": UID_A, "namespace": "ns", "name": "p", "containers": {}}})
    cp = ControlPlane([_Static(md), _Boom()], interval=0.05)
    cp.attach(e)
    cp.refresh_once()
    assert cp.last_complete is False

    def energy():
        f = promtext.parse(e.snapshot_text())
        return {s[1]["pod"]: s[2] for s in promtext.samples(f, "amd_pod_gpu_energy_joules_total")}
    e.tick(1_000_000_000)
    e.tick(2_000_000_000)
    assert energy() == {"gone": 123, "p": 7}
    assert promtext.value(promtext.parse(e.snapshot_text()), "amd_pod_xgmi_write_bytes_total", pod="gone") == 2000
    cp.sources = [_Static(md)]  # the apiserver is back: a complete refresh
    cp.refresh_once()
    assert cp.last_complete is True
    e.tick(3_000_000_000)
    assert energy() == {"p": 7}
    assert "amd_pod_xgmi_write_bytes_total" not in e.snapshot_text()


def test_full_exporter_on_fake_node(tmp_path):
    """sysfs backend + fake kubelet + fake apiserver, through the Exporter/Config path."""
    import shutil
    import tempfile
    from pathlib import Path

    from kubernetes_gpu_exporter_amd.exporter import Exporter
    root = Path(tempfile.mkdtemp(prefix="h", dir="/tmp"))  # unix socket paths max 107 chars
    request_cleanup = lambda: shutil.rmtree(root, ignore_errors=True)  # noqa: E731
    h = mi355x_node(root, 3)  # GPUs at 0a (idx0), 5a (idx1), 72 (idx2)
    by_bus = {g.location_id >> 8: g for g in h.gpus}
    h.add_process(1001, kubepods_cgroup(UID_A, CID_A), gpus={by_bus[0x72].gpu_id: (40 << 30, 200)})
    h.add_process(1002, kubepods_cgroup(UID_B, CID_B, qos="guaranteed"), gpus={by_bus[0x5A].gpu_id: (20 << 30, 100)})
    sock_rel = "/var/lib/kubelet/pod-resources/kubelet.sock"
    kub = FakeKubelet(str(root) + sock_rel, pods(), node="node-a").start()
    api = FakeApiserver(pods(), token="tok").start()
    (tmp_path / "token").write_text("tok")
    cfg = make_config({"backend": "sysfs", "host_root": str(root), "interval": 0, "listen": "127.0.0.1:0",
                       "node_name": "node-a", "apiserver": api.url, "apiserver_token_file": str(tmp_path / "token"),
                       "kubelet_socket": sock_rel, "control_interval": 0.05})
    ex = Exporter(cfg)
    try:
        ex.start()
        srcs = {s.name for s in ex._control.sources}
        assert srcs == {"apiserver", "podresources"}, srcs
        ex.tick(1_000_000_000)
        ex.tick(1_100_000_000)
        fams = promtext.parse(ex.text())
        assert promtext.value(fams, "pod_gpu_memory_usage", pid=1001, pod="llama-train-0") == 40 << 30
        assert promtext.value(fams, "pod_gpu_memory_usage", pid=1002, pod="vllm-0") == 20 << 30
        up = {s[1]["bdf"]: s[1] for s in fams["amd_gpu_up"].samples}
        assert (up["0000:72:00.0"]["namespace"], up["0000:72:00.0"]["pod"]) == ("research", "llama-train-0")
        assert up["0000:5a:00.0"]["container"] == "server"
        assert up["0000:23:00.0"]["pod"] == ""  # its pod runs on node-b: not ours
        assert promtext.value(fams, "amd_pod_gpus", pod="vllm-0") == 1
        assert promtext.value(fams, "amd_gpu_process_vram_bytes", pid=1002, container="server") == 20 << 30
        # apiserver outage: last known metadata keeps attribution working
        api.fail_status = 503
        assert _wait(lambda: ex._control.refresh_once() is not None and "apiserver" in ex._control.errors)
        ex.tick(10_000_000_000)
        fams = promtext.parse(ex.text())
        assert promtext.value(fams, "pod_gpu_memory_usage", pid=1002, pod="vllm-0") == 20 << 30
    finally:
        ex.stop()
        kub.stop()
        api.stop()
        request_cleanup()


def _wait(pred, timeout=5.0):
    import time
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_apiserver_list_then_watch(tmp_path):
    """One list, then events over a single watch: refreshes cost no requests; ADDED /
    MODIFIED / DELETED land in the cache; other nodes' events are filtered server-side."""
    api = FakeApiserver(pods(), token="").start()
    src = ApiserverSource(api.url, "node-a", "", watch_timeout_s=30)
    try:
        assert set(src.fetch().pods) == {UID_A, UID_B}
        assert _wait(lambda: any("watch=1" in r for r in api.requests))
        n_req = len(api.requests)
        new_uid = "99999999-8888-7777-6666-555555555555"
        api.add_pod(FakePod(new_uid, "team", "late-pod", node="node-a", containers={"c": "e" * 64}))
        api.add_pod(FakePod("11111111-0000-0000-0000-000000000000", "x", "elsewhere", node="node-b"))
        assert _wait(lambda: new_uid in src.fetch().pods)
        assert src.fetch().pods[new_uid]["containers"] == {"e" * 64: "c"}
        api.update_pod(FakePod(new_uid, "team", "late-pod", node="node-a", containers={"c": "f" * 64}))
        assert _wait(lambda: src.fetch().pods[new_uid]["containers"] == {"f" * 64: "c"})
        api.delete_pod(UID_A)
        assert _wait(lambda: UID_A not in src.fetch().pods)
        assert "11111111-0000-0000-0000-000000000000" not in src.fetch().pods
        for _ in range(20):
            src.fetch()
        assert len(api.requests) == n_req  # every refresh above was served from the cache
        assert src.relists == 1
    finally:
        src.close()
        api.stop()


def test_apiserver_watch_resumes_and_relists_on_410(tmp_path):
    api = FakeApiserver(pods(), token="").start()
    src = ApiserverSource(api.url, "node-a", "", watch_timeout_s=1)  # server ends each watch after 1 s
    try:
        src.fetch()
        assert _wait(lambda: sum("watch=1" in r for r in api.requests) >= 2, timeout=6)  # resumed
        assert src.relists == 1
        api.expire_before = api.rv + 100          # history compacted: next resume gets 410
        api.bookmark()
        assert _wait(lambda: src.relists >= 2, timeout=6)
        api.expire_before = 0
        late = "abababab-0000-0000-0000-000000000000"
        api.add_pod(FakePod(late, "ns", "after-relist", node="node-a"))
        assert _wait(lambda: late in src.fetch().pods, timeout=6)
    finally:
        src.close()
        api.stop()


def test_apiserver_outage_keeps_cache_and_recovers(tmp_path):
    api = FakeApiserver(pods(), token="").start()
    src = ApiserverSource(api.url, "node-a", "", watch_timeout_s=1)
    try:
        src.fetch()
        api.fail_status = 503
        import time
        time.sleep(1.5)                           # watch ends, reconnects fail with 503
        assert set(src.fetch().pods) == {UID_A, UID_B}  # stale cache, not an empty map
        api.fail_status = 0
        late = "cdcdcdcd-0000-0000-0000-000000000000"
        api.add_pod(FakePod(late, "ns", "after-outage", node="node-a"))
        assert _wait(lambda: late in src.fetch().pods, timeout=10)
    finally:
        src.close()
        api.stop()


@pytest.mark.parametrize("xcp_files", [True, False])
def test_cpx_partitions_owned_by_eight_pods(tmp_path, xcp_files):
    """A CPX-mode MI355X socket: 8 logical GPUs with ONE PCI BDF, each allocated to its own
    pod by the device plugin (partition-mode resource amd.com/cpx_nps4; partition 0 named
    by the BDF, the others by their XCP platform devices).  Every logical GPU's device
    series must carry its own pod — keyed by BDF alone they would all collapse to one."""
    import shutil
    import tempfile
    from pathlib import Path

    from kubernetes_gpu_exporter_amd.exporter import Exporter
    from kubernetes_gpu_exporter_amd.utils.fakehost import mi355x_cpx_socket
    root = Path(tempfile.mkdtemp(prefix="c", dir="/tmp"))
    try:
        h = mi355x_cpx_socket(root, xcp_files=xcp_files)
        for g in h.gpus:
            h.set_metrics(g, gfx=50, num_partition=8)
        ids = ["0000:72:00.0"] + [f"amdgpu_xcp_{k}" for k in range(1, 8)]
        cpods = [FakePod(f"{k:08x}-0000-4000-8000-00000000000{k}", "infer", f"shard-{k}", "node-a",
                         {"srv": f"{k:02x}" * 32}, {"srv": [ids[k]]}) for k in range(8)]
        sock_rel = "/var/lib/kubelet/pod-resources/kubelet.sock"
        kub = FakeKubelet(str(root) + sock_rel, cpods, resource="amd.com/cpx_nps4", node="node-a").start()
        cfg = make_config({"backend": "sysfs", "host_root": str(root), "interval": 0, "listen": "127.0.0.1:0",
                           "node_name": "node-a", "kubelet_socket": sock_rel, "control_interval": 0.05,
                           "series_profile": "full"})
        ex = Exporter(cfg)
        try:
            ex.start()
            ex.tick(1_000_000_000)
            ex.tick(1_100_000_000)
            fams = promtext.parse(ex.text())
            up = {s[1]["gpu"]: s[1] for s in fams["amd_gpu_up"].samples}
            assert {g: (l["namespace"], l["pod"], l["container"]) for g, l in up.items()} == \
                {str(k): ("infer", f"shard-{k}", "srv") for k in range(8)}
            info = {s[1]["gpu"]: s[1] for s in fams["amd_gpu_info"].samples}
            assert [info[str(k)]["device_node"] for k in range(8)] == ["0000:72:00.0"] + \
                [f"amdgpu_xcp.{k}" for k in range(1, 8)]
            assert {s[1]["bdf"] for s in fams["amd_gpu_up"].samples} == {"0000:72:00.0"}
            # socket telemetry read from the PCI function for every partition
            assert {s[2] for s in fams["amd_gpu_up"].samples} == {1.0}
            assert all(promtext.value(fams, "amd_pod_gpus", pod=f"shard-{k}") == 1 for k in range(8))
        finally:
            ex.stop()
            kub.stop()
    finally:
        shutil.rmtree(root, ignore_errors=True)


def test_partition_owner_keys(native, tmp_path):
    """Which device-plugin ids name which logical GPU: the bare BDF names partition 0 only;
    XCP names (both spellings), <bdf>/<k>, render nodes, kfd:<id> and UUIDs each name one."""
    from kubernetes_gpu_exporter_amd.utils.fakehost import mi355x_cpx_socket
    h = mi355x_cpx_socket(tmp_path, partitions=4)
    devs = native.read_backend("sysfs", str(tmp_path))
    keys = [d["owner_keys"] for d in devs]
    assert "0000:72:00.0" in keys[0] and all("0000:72:00.0" not in k for k in keys[1:])
    for k in range(1, 4):
        assert {f"amdgpu_xcp.{k}", f"amdgpu_xcp_{k}", f"0000:72:00.0/{k}", f"renderd{128 + k}",
                f"/dev/dri/renderd{128 + k}", f"kfd:{h.gpus[k].gpu_id}"} <= set(keys[k])
    flat = [x for ks in keys for x in ks if not x.startswith("e2")]  # UUIDs: shared unique_id in the fixture
    assert len(flat) == len(set(flat))  # no id names two logical GPUs
