"""Synthetic pod workloads (models/): every strategy runs across 2 gloo ranks on CPU and
reports the per-op payload the RCCL tracer must see; GemmPod math matches fp32."""
import json
import os
import subprocess
import sys

import pytest
import torch

from kubernetes_gpu_exporter_amd.models import WORKLOADS, GemmPod, make, run
from kubernetes_gpu_exporter_amd.parallel.launch import spawn, workload_worker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gemm_pod_cpu_math():
    p = GemmPod(size=64, iters=1, device="cpu")
    s = p.step()
    assert s.flops == 2 * 64 ** 3
    torch.testing.assert_close(p.c, p.a @ p.b.T)


def test_unknown_workload_rejected():
    with pytest.raises(ValueError):
        make("zz")


@pytest.mark.parametrize("name", [w for w in WORKLOADS if w != "gemm"])
def test_trainer_pods_two_ranks(name):
    kw = {"size": 32, "iters": 1, "comm_bytes": 1 << 14, "device": "cpu"}
    res = spawn(workload_worker, 2, "gloo", args=(name, 3, kw))
    assert [r["workload"] for r in res] == [name, name]
    for rank, r in enumerate(res):
        assert r["steps"] == 3 and r["tflops"] > 0
        if name == "pp":  # rank 0 only sends, the last rank only receives
            assert set(r["comm_bytes"]) == ({"send"} if rank == 0 else {"recv"})
        else:
            assert r["comm_bytes"] and all(v > 0 for v in r["comm_bytes"].values())
    if name == "dp":
        assert res[0]["comm_calls"] == {"allreduce": 3}
        assert res[0]["comm_bytes"]["allreduce"] == 3 * (1 << 14)


def test_models_cli_single_process():
    r = subprocess.run([sys.executable, "-m", "kubernetes_gpu_exporter_amd.models", "gemm", "--steps", "2",
                        "--warmup", "0", "--size", "64", "--iters", "1"], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["workload"] == "gemm" and out["steps"] == 2
