"""RCCL tracer shared-memory protocol (csrc/gpuexp/rccl_shm.h) -> per-pod collective
series, without a GPU: the test plays the tracer's role and writes the file itself."""
import mmap
import os
import struct

from kubernetes_gpu_exporter_amd.utils import promtext

MAGIC = 0x3158455550474D52
OPS = ["allreduce", "allgather", "reducescatter", "alltoall", "alltoallv", "broadcast", "reduce",
       "send", "recv", "gather", "scatter"]
SIZE = 64 + 16 * 16
UID = "12345678-1234-1234-1234-123456789abc"
CG = "/kubepods/burstable/pod" + UID + "/" + "b" * 64


def write_shm(path, ns_pid, ops):
    with open(path, "wb") as fh:
        fh.write(b"\0" * SIZE)
    fd = os.open(path, os.O_RDWR)
    m = mmap.mmap(fd, SIZE)
    os.close(fd)
    struct.pack_into("<QIiQii", m, 0, 0, 1, ns_pid, os.stat("/proc/self/ns/pid").st_ino, 0, 4)
    for name, (calls, nbytes) in ops.items():
        struct.pack_into("<QQ", m, 64 + 16 * OPS.index(name), calls, nbytes)
    struct.pack_into("<Q", m, 0, MAGIC)  # publish
    return m


def test_rccl_counters_attributed_to_pod(mock_engine, tmp_path):
    d = tmp_path / "rccl"
    d.mkdir()
    pid = 31337
    m = write_shm(str(d / f"gpuexp-rccl-1-{pid}"), pid, {"allreduce": (10, 10 * 64 << 20), "send": (3, 3000)})
    e = mock_engine(1, http=False, enable_rccl=True, rccl_dir=str(d))
    e.set_pid_cgroup(pid, CG)
    e.set_pods([dict(uid=UID, namespace="train", name="dp-worker-0", containers={})])
    e.tick(1_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "amd_rccl_collective_calls_total", pod="dp-worker-0", op="allreduce") == 10
    assert promtext.value(fams, "amd_rccl_collective_bytes_total", namespace="train", op="allreduce",
                          pid=pid) == 10 * 64 << 20
    assert promtext.value(fams, "amd_rccl_collective_calls_total", op="send") == 3
    # rank / size of the process's communicator (the file says rank 0 of 4)
    assert promtext.value(fams, "amd_rccl_communicator_info", pod="dp-worker-0", rank=0, nranks=4) == 1
    # the tracer keeps counting; the exporter reads the live mapping
    struct.pack_into("<QQ", m, 64, 25, 25 * 64 << 20)
    e.tick(2_000_000_000)
    fams = promtext.parse(e.snapshot_text())
    assert promtext.value(fams, "amd_rccl_collective_calls_total", op="allreduce") == 25
    # process gone (file unlinked by the tracer at exit) -> series vanish
    os.unlink(d / f"gpuexp-rccl-1-{pid}")
    e.tick(3_000_000_000)
    assert "amd_rccl_collective_calls_total" not in e.snapshot_text()


def test_incomplete_file_ignored(mock_engine, tmp_path):
    (tmp_path / "gpuexp-rccl-1-5").write_bytes(b"\0" * 10)  # truncated
    full = write_shm(str(tmp_path / "gpuexp-rccl-1-6"), 6, {"alltoall": (1, 8)})
    struct.pack_into("<Q", full, 0, 0)  # magic not yet published
    e = mock_engine(1, http=False, enable_rccl=True, rccl_dir=str(tmp_path))
    e.tick(1)
    assert "amd_rccl" not in e.snapshot_text()
