"""Multi-node tier: several exporter instances, each on its own fake
host root (8 MI355X GPUs, KFD process files, cgroups) with its own kubelet PodResources
socket and NODE_NAME, sharing one fake apiserver whose pods are spread over the nodes.
One harness scrapes every instance over real HTTP the way Prometheus does (adding an
`instance` label) and checks the federated view: every pod is reported by exactly the
node it runs on, device ownership follows the device plugin, and losing one node's
exporter leaves the others untouched.

The reference listed every pod of the whole cluster from every node (`main.go:77`) and
keyed its map by pod name only (`main.go:113`); both would double-count here.
"""
import shutil
import tempfile
import time
import urllib.request
from pathlib import Path

import pytest

from kubernetes_gpu_exporter_amd.config import make_config
from kubernetes_gpu_exporter_amd.exporter import Exporter
from kubernetes_gpu_exporter_amd.k8s.fakes import FakeApiserver, FakeKubelet, FakePod
from kubernetes_gpu_exporter_amd.utils import promtext
from kubernetes_gpu_exporter_amd.utils.fakehost import kubepods_cgroup, mi355x_node

NODES = ("node-a", "node-b")
GPUS = 8
SOCK = "/var/lib/kubelet/pod-resources/kubelet.sock"


def _uid(node: int, k: int) -> str:
    return f"{node:08x}-0000-4000-8000-{k:012d}"


def _cid(node: int, k: int) -> str:
    return f"{node:02x}{k:02x}" * 16


def _build_cluster(roots):
    """Per node: one single-GPU training pod per GPU (same pod NAMES on both nodes, in
    different namespaces) plus an inference pod sharing GPU 0 without a device grant."""
    pods, hosts = [], []
    for n, (node, root) in enumerate(zip(NODES, roots)):
        h = mi355x_node(root, GPUS)
        hosts.append(h)
        bdfs = [f"0000:{g.location_id >> 8:02x}:00.0" for g in h.gpus]
        for k, g in enumerate(h.gpus):
            uid, cid = _uid(n, k), _cid(n, k)
            pods.append(FakePod(uid, f"team-{n}", f"train-{k}", node, {"trainer": cid}, {"trainer": [bdfs[k]]}))
            h.add_process(10_000 * (n + 1) + k, kubepods_cgroup(uid, cid, qos="guaranteed"),
                          gpus={g.gpu_id: ((k + 1) << 30, 50)})
        uid, cid = _uid(n, 99), _cid(n, 99)
        pods.append(FakePod(uid, f"team-{n}", "infer", node, {"server": cid}))
        h.add_process(10_000 * (n + 1) + 99, kubepods_cgroup(uid, cid), gpus={h.gpus[0].gpu_id: (512 << 20, 10)})
    return pods, hosts


def _scrape(port: int) -> dict:
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
        assert r.status == 200
        return promtext.parse(r.read().decode())


def _federate(scrapes: dict) -> list:
    """Prometheus-style merge: every sample gets the instance label of its target."""
    out = []
    for inst, fams in scrapes.items():
        for fam in fams.values():
            for name, lab, v in fam.samples:
                out.append((name, dict(lab, instance=inst), v))
    return out


def _wait(pred, timeout=10.0):
    t = time.monotonic() + timeout
    while time.monotonic() < t:
        if pred():
            return True
        time.sleep(0.05)
    return False


@pytest.fixture
def cluster(tmp_path):
    roots = [Path(tempfile.mkdtemp(prefix="mn", dir="/tmp")) for _ in NODES]  # short unix socket paths
    pods, hosts = _build_cluster(roots)
    api = FakeApiserver(pods, token="tok").start()
    (tmp_path / "token").write_text("tok")
    kubelets, exporters = [], {}
    try:
        for node, root in zip(NODES, roots):
            kubelets.append(FakeKubelet(str(root) + SOCK, pods, node=node).start())
            cfg = make_config({"backend": "sysfs", "host_root": str(root), "interval": 0.05,
                               "listen": "127.0.0.1:0", "node_name": node, "apiserver": api.url,
                               "apiserver_token_file": str(tmp_path / "token"), "kubelet_socket": SOCK,
                               "control_interval": 0.05})
            exporters[node] = Exporter(cfg).start()
        yield {"pods": pods, "hosts": hosts, "api": api, "exporters": exporters}
    finally:
        for ex in exporters.values():
            ex.stop()
        for k in kubelets:
            k.stop()
        api.stop()
        for r in roots:
            shutil.rmtree(r, ignore_errors=True)


def _attributed(ex) -> bool:
    """Both control-plane inputs have arrived: pod names (apiserver, for the PID -> pod
    join) and device grants (kubelet PodResources, for GPU -> owner)."""
    fams = _scrape(ex.port)
    procs_ok = len({lab["pod"] for _, lab, _ in promtext.samples(fams, "pod_gpu_memory_usage")}) == GPUS + 1
    owners_ok = all(lab["pod"] for _, lab, _ in promtext.samples(fams, "amd_gpu_up"))
    return procs_ok and owners_ok


def test_each_node_reports_only_its_own_pods(cluster):
    exs = cluster["exporters"]
    assert all(_wait(lambda ex=ex: _attributed(ex)) for ex in exs.values())
    fed = _federate({node: _scrape(ex.port) for node, ex in exs.items()})

    # device series: 2 nodes x 8 GPUs, each GPU owned by the pod the device plugin gave it
    # (the exporter numbers GPUs by PCI BDF; the fixture's k-th GPU is the k-th bus it made)
    k_of_bdf = {f"0000:{g.location_id >> 8:02x}:00.0": k for k, g in enumerate(cluster["hosts"][0].gpus)}
    up = [(lab, v) for name, lab, v in fed if name == "amd_gpu_up"]
    assert len(up) == len(NODES) * GPUS and all(v == 1 for _, v in up)
    for lab, _ in up:
        n = NODES.index(lab["instance"])
        assert lab["namespace"] == f"team-{n}" and lab["pod"] == f"train-{k_of_bdf[lab['bdf']]}", lab

    # per-process series: each host PID once, on its own node, with its pod and namespace
    vram = {(lab["instance"], int(lab["pid"])): (lab, v) for name, lab, v in fed
            if name == "amd_gpu_process_vram_bytes"}
    assert len(vram) == len(NODES) * (GPUS + 1)
    for (inst, pid), (lab, v) in vram.items():
        n = NODES.index(inst)
        assert pid // 10_000 == n + 1, (inst, pid)        # never another node's process
        k = pid % 10_000
        assert lab["namespace"] == f"team-{n}"
        assert lab["pod"] == ("infer" if k == 99 else f"train-{k}")
        assert v == (512 << 20 if k == 99 else (k + 1) << 30)

    # legacy families: same pod names exist on both nodes; per instance they never collide
    legacy = [(lab, v) for name, lab, v in fed if name == "pod_gpu_memory_usage"]
    assert len(legacy) == len(NODES) * (GPUS + 1)
    for n, node in enumerate(NODES):
        mine = {lab["pod"]: v for lab, v in legacy if lab["instance"] == node}
        assert mine == {**{f"train-{k}": float((k + 1) << 30) for k in range(GPUS)}, "infer": float(512 << 20)}

    # the shared first GPU carries two processes (two pods), the others one each
    procs = {(lab["instance"], k_of_bdf[lab["bdf"]]): v for name, lab, v in fed if name == "amd_gpu_processes"}
    for node in NODES:
        assert procs[(node, 0)] == 2 and all(procs[(node, k)] == 1 for k in range(1, GPUS))


def test_node_loss_leaves_other_nodes_intact(cluster):
    exs = cluster["exporters"]
    assert all(_wait(lambda ex=ex: _attributed(ex)) for ex in exs.values())
    port_b = exs["node-b"].port
    exs["node-b"].stop()
    with pytest.raises(OSError):
        _scrape(port_b)
    # node-a keeps sampling: its tick counter still advances and its pods stay attributed
    t0 = promtext.value(_scrape(exs["node-a"].port), "gpuexp_ticks_total")
    assert _wait(lambda: promtext.value(_scrape(exs["node-a"].port), "gpuexp_ticks_total") > t0 + 2)
    assert _attributed(exs["node-a"])


def test_pod_moves_between_nodes(cluster):
    """A pod rescheduled to the other node (new UID, same name) is reported by the new
    node only, and the old node drops its series once its process is gone."""
    exs, hosts, api = cluster["exporters"], cluster["hosts"], cluster["api"]
    assert all(_wait(lambda ex=ex: _attributed(ex)) for ex in exs.values())
    # node-a's infer pod dies ...
    hosts[0].remove_process(10_000 + 99)
    api.delete_pod(_uid(0, 99))
    # ... and comes back on node-b as a second inference replica under team-0
    uid, cid = "feedface-0000-4000-8000-000000000001", "fe" * 32
    api.add_pod(FakePod(uid, "team-0", "infer", "node-b", {"server": cid}))
    hosts[1].add_process(20_099 + 1, kubepods_cgroup(uid, cid), gpus={hosts[1].gpus[3].gpu_id: (1 << 30, 5)})

    def moved():
        a = _scrape(exs["node-a"].port)
        b = _scrape(exs["node-b"].port)
        a_inf = [lab for _, lab, _ in promtext.samples(a, "amd_gpu_process_vram_bytes") if lab["pod"] == "infer"]
        b_inf = {(lab["namespace"], lab["pid"]) for _, lab, _ in promtext.samples(b, "amd_gpu_process_vram_bytes")
                 if lab["pod"] == "infer"}
        return not a_inf and b_inf == {("team-1", "20099"), ("team-0", "20100")}
    assert _wait(moved), (_scrape(exs["node-b"].port).get("amd_gpu_process_vram_bytes"))
