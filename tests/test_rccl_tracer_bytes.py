"""Byte accounting of the RCCL tracer (csrc/gpuexp/rccl_tracer.cc) for every op at
nranks > 1, without a GPU: csrc/tests/rccl_tracer_test.cc feeds the tool's rocprofiler
callback synthetic API records (a communicator of N ranks, then one call of each op,
an all-to-all whose RCCL-internal send/recv are nested inside it, and a communicator the
tool never saw created) and the resulting shared-memory counters are checked against the
formulas of the tracer's header comment, the same ones parallel/collectives.py's
TrafficStats uses for the generators."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BF16 = 2


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not shutil.which("g++") or not os.path.exists("/opt/rocm/include/rocprofiler-sdk/rccl/api_args.h"):
        pytest.skip("needs g++ and the rocprofiler-sdk headers")
    out = tmp_path_factory.mktemp("rt") / "rccl_tracer_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "csrc"), "-I/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "csrc/tests/rccl_tracer_test.cc"), "-o", str(out),
                    "-ldl", "-lpthread", "-Wl,--unresolved-symbols=ignore-in-object-files"],
                   check=True, capture_output=True, text=True)
    return str(out)


def run(harness, tmp_path, nranks, rank, count):
    r = subprocess.run([harness, str(tmp_path), str(nranks), str(rank), str(count)], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("nranks,rank", [(8, 3), (2, 1), (1, 0)])
def test_every_op_byte_formula(harness, tmp_path, nranks, rank):
    count = 1000
    d = run(harness, tmp_path, nranks, rank, count)
    assert d["rank"] == rank and d["nranks"] == nranks
    ops = {k: tuple(v) for k, v in d["ops"].items()}
    n = count * BF16
    want = {
        "allreduce": (1, n),                          # count * size
        "allgather": (2, n * nranks + count * 4),      # sendcount * size * nranks (+ unknown comm: x1, fp32)
        "reducescatter": (1, n * nranks),              # recvcount * size * nranks
        "alltoall": (1, n * nranks),                   # count (per peer) * size * nranks; nested send/recv not counted
        "alltoallv": (1, (nranks * count + nranks * (nranks - 1) // 2) * BF16),  # sum(sendcounts) * size
        "broadcast": (1, n),
        "reduce": (1, n),
        "send": (1, n),                                # PP / CP point-to-point: count * size
        "recv": (1, n),
        "gather": (1, n),                              # this rank's contribution: sendcount * size
        "scatter": (1, n),                             # recvcount * size
    }
    assert ops == want


def test_file_identity_and_cleanup(harness, tmp_path):
    d = run(harness, tmp_path, 4, 2, 16)
    name = os.path.basename(d["path"])
    ino = os.stat("/proc/self/ns/pid").st_ino
    assert name.startswith(f"gpuexp-rccl-{ino}-")  # <pidns inode>-<pid in that namespace>
    assert os.path.exists(d["path"])  # GPUEXP_RCCL_KEEP: left for inspection
