"""cgroup path corpus: systemd / cgroupfs drivers x containerd / cri-o / docker x QoS
classes, plus nested (kind / k3s-in-docker) and non-kube paths.  This replaces the
reference's `kubectl exec <pod> -- ps` PID discovery (/root/reference/main.go:101)."""
import pytest

UID = "0a1b2c3d-4e5f-6789-abcd-ef0123456789"
U_ = UID.replace("-", "_")
CID = "4f3c2b1a" * 8

CASES = [
    # (path, qos, runtime)
    (f"/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{U_}.slice/cri-containerd-{CID}.scope",
     "burstable", "containerd"),
    (f"/kubepods.slice/kubepods-besteffort.slice/kubepods-besteffort-pod{U_}.slice/crio-{CID}.scope",
     "besteffort", "crio"),
    (f"/kubepods.slice/kubepods-pod{U_}.slice/docker-{CID}.scope", "guaranteed", "docker"),
    (f"/kubepods/burstable/pod{UID}/{CID}", "burstable", "unknown"),
    (f"/kubepods/pod{UID}/{CID}", "guaranteed", "unknown"),
    (f"/kubepods/besteffort/pod{UID}/{CID}", "besteffort", "unknown"),
    # kind (systemd inside a node container)
    (f"/kubelet.slice/kubelet-kubepods.slice/kubelet-kubepods-besteffort.slice/"
     f"kubelet-kubepods-besteffort-pod{U_}.slice/cri-containerd-{CID}.scope", "besteffort", "containerd"),
    # k3s / docker-in-docker nesting
    (f"/docker/{'e' * 64}/kubepods/burstable/pod{UID}/{CID}", "burstable", "unknown"),
    # containerd systemd cgroup with ":" separators
    (f"/system.slice/containerd.service/kubepods-burstable-pod{U_}.slice:cri-containerd:{CID}",
     "burstable", "containerd"),
]


@pytest.mark.parametrize("path,qos,runtime", CASES)
def test_kube_paths(native, path, qos, runtime):
    r = native.parse_cgroup_path(path)
    assert r["kube"] is True
    assert r["pod_uid"] == UID
    assert r["container_id"] == CID
    assert r["qos"] == qos
    assert r["runtime"] == runtime


def test_pod_level_process_without_container(native):
    r = native.parse_cgroup_path(f"/kubepods/burstable/pod{UID}")
    assert r["kube"] and r["pod_uid"] == UID and r["container_id"] == ""


def test_crio_conmon_is_not_a_container(native):
    r = native.parse_cgroup_path(
        f"/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{U_}.slice/crio-conmon-{CID}.scope")
    assert r["kube"] and r["container_id"] == ""


@pytest.mark.parametrize("path", [
    "/", "/user.slice/user-1000.slice/session-1.scope", "/system.slice/docker.service",
    "/process_api/b56d38b91ace84d497a7f126f1c246f8",  # the GPU box's own cgroup
    "/kubepods.slice", "/kubepods/burstable/podnot-a-uid/abc",
])
def test_non_kube_paths(native, path):
    assert native.parse_cgroup_path(path)["kube"] is False


def test_proc_cgroup_v2_and_v1(native):
    v2 = f"0::/kubepods/pod{UID}/{CID}\n"
    assert native.parse_proc_cgroup(v2)["pod_uid"] == UID
    v1 = ("12:pids:/kubepods/burstable/pod%s/%s\n11:memory:/kubepods/burstable/pod%s/%s\n"
          "1:name=systemd:/kubepods/burstable/pod%s/%s\n" % ((UID, CID) * 3))
    r = native.parse_proc_cgroup(v1)
    assert r["kube"] and r["container_id"] == CID
    assert native.parse_proc_cgroup("0::/init.scope\n")["kube"] is False


def test_uppercase_uid_is_normalised(native):
    r = native.parse_cgroup_path(f"/kubepods/pod{UID.upper()}/{CID}")
    assert r["pod_uid"] == UID
