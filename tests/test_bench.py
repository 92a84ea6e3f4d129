"""bench.py contract (the driver's launch lines), on CPU with the mock backend:
one JSON line from rank 0 with the required keys, single-process and under torchrun."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(stdout):
    out = []
    for line in stdout.splitlines():
        line = line.strip()
        if line.startswith("{"):
            out.append(json.loads(line))
    return out


def _check(d, n, steps, warmup):
    assert KEYS <= set(d), KEYS - set(d)
    assert d["n_gpus"] == n and d["steps"] == steps and d["warmup"] == warmup
    assert d["higher_is_better"] is False and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    assert d["config"]["parallelism"] == f"dp{n}"
    assert d["scrapes"] == steps and d["scrape_errors"] == 0
    assert all(v >= 64 for v in d["series_per_gpu"].values()), d["series_per_gpu"]


def test_bench_single_process():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "1", "--backend", "mock"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    _check(d, 1, 5, 1)
    # Native libraries (RCCL's banner) and the exporter child write to stderr only.
    assert r.stdout.strip().count("\n") == 0, r.stdout[-2000:]


def test_bench_torchrun_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 only
    _check(lines[0], 2, 4, 1)
    assert lines[0]["attributed_pods"] == ["gemm-pod-0", "gemm-pod-1"] or lines[0]["config"]["backend"] == "mock"
