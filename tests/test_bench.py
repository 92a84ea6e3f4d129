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
    # where the exporter's CPU went, per thread name, and its KFD scans (diagnostics)
    assert d["exporter_cpu_us_per_step_by_thread"].get("gpuexp-sampler", 0) > 0, d["exporter_cpu_us_per_step_by_thread"]
    assert set(d["kfd_proc_scans"]) == {"list", "tracked"} and d["kfd_procs_tracked"] >= 1, d
    assert d["http_rx_cpu_moves"] == 0  # follow_rx_cpu is off by default
    # Native libraries (RCCL's banner) and the exporter child write to stderr only.
    assert r.stdout.strip().count("\n") == 0, r.stdout[-2000:]


def test_bench_self_launches_one_rank_per_gpu():
    """`bench.py --gpus 4` with no launcher starts 4 ranks itself (gloo on CPU): 4 mock
    GPUs, 4 GEMM pods attributed through the KFD reader + pod map, one result line."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--backend", "mock", "--steps", "4", "--warmup",
                        "1"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    _check(d, 4, 4, 1)
    assert d["ranks"] == 4 and d["config"]["global_batch"] == 4
    assert d["attributed_pods"] == [f"gemm-pod-{i}" for i in range(4)]
    assert sorted(d["series_per_gpu"]) == ["0", "1", "2", "3"]
    assert d["p99_scrape_us"] is None  # 4 samples: no p99 claimed
    assert d["server_scrapes"] >= 3 and d["server_scrape_p99_le_us"] > 0
    assert d["sampler_cpu_us_per_tick_per_gpu"] > 0 and d["exporter_rss_mb"] > 0
    assert "measured_over_expected_write" in d["xgmi_timed_window"]
    assert "rccl_files" in d  # tracer file states (None on the mock backend: no tracer)
    # untimed pattern phase: ring + all-to-all ran on all ranks; per-rank link bytes are
    # joined to peer ranks through the peer_bdf labels (mock links: synthetic bytes)
    pat = d["xgmi_patterns"]
    assert set(pat) == {"cp", "ep"}, pat
    for p in pat.values():
        assert p["steps"] >= 1 and sorted(p["per_rank"]) == ["0", "1", "2", "3"]
        assert p["expected_bytes_out_per_rank"] > 0
        peers = set(p["per_rank"]["0"]["per_peer_share"])
        assert {"1", "2", "3"} <= peers, peers  # mock GPU 0's links to mock GPUs 1..3 resolve to ranks


def test_bench_world_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--backend", "mock", "--steps", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
    assert not _json_lines(r.stdout)


def test_bench_failed_rank_stops_the_job():
    env = dict(os.environ, GPUEXP_BENCH_FAIL_RANK="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "mock", "--steps", "50"], cwd=ROOT,
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "rank 1 exited with 3" in r.stderr


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


def test_bench_eight_ranks_every_check_holds():
    """The driver's 8-GPU shape, rehearsed on CPU (8 gloo ranks, 8 mock GPUs): one line,
    every GPU exported, every rank's pod attributed, and the run's own validity checks
    (bench.run_problems) empty; the timed scrapes are each accounted pre-woken or not.  The
    xGMI pattern phase runs too: the ranks' ring (CP) and all-to-all (EP) traffic per peer
    reaches the mock GPUs' links (MockBackend::set_traffic_file), and the exporter's per-peer
    attribution must show it: every rank's ring-neighbour share >= 0.9, every all-to-all
    peer share within 20 % of uniform (result['xgmi_checks'])."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--backend", "mock", "--steps", "4", "--warmup",
                        "1"], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    _check(d, 8, 4, 1)
    assert sorted(d["series_per_gpu"], key=int) == [str(i) for i in range(8)]
    assert d["attributed_pods"] == sorted(f"gemm-pod-{i}" for i in range(8))
    assert 0 < d["exporter_startup_s"] <= d["exporter_startup_budget_s"]
    pw = d["prewake"]
    assert pw["timed_scrapes"] == 4 and pw["prewoken"] + pw["not_prewoken"] + pw["unknown"] == 4, pw
    assert pw["unknown"] == 0, pw  # the server echoes the pre-wake state of every timed scrape
    chk = d["xgmi_checks"]
    assert chk["cp_ok"] and chk["cp_ring_neighbour_share_min"] >= 0.9, (chk, d["xgmi_patterns"]["cp"])
    assert chk["ep_ok"] and chk["ep_max_deviation_from_uniform"] <= 0.2, (chk, d["xgmi_patterns"]["ep"])
    assert chk["dp_ok"] is None  # the DP all-reduce's per-peer split is RCCL's: nothing injected on mock links
    for r_, v in d["xgmi_patterns"]["cp"]["per_rank"].items():
        nbr = {str((int(r_) + 1) % 8), str((int(r_) - 1) % 8)}
        assert set(k for k, x in v["per_peer_share"].items() if x > 0.01) <= nbr, (r_, v)


def test_bench_unattributed_rank_fails_loudly():
    """At N > 1 a rank whose pod never attributes makes the run invalid: exit 1, no result
    line (a degraded configuration must not reach SCALE as a number)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", GPUEXP_BENCH_NO_POD_RANK="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--backend", "mock", "--steps", "3", "--warmup",
                        "1", "--xgmi-patterns", "0"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "FAILED: attributed pods" in r.stderr, r.stderr[-2000:]


def test_bench_degraded_single_gpu_run_fails_loudly():
    """At N = 1 too: an exporter that only starts without the PMC counters and the sentinel is
    a degraded configuration -> exit 1, no result line, the reason on stderr (round 3 printed
    the headline anyway)."""
    env = dict(os.environ, GPUEXP_BENCH_FAIL_EXPORTER_WITH_COUNTERS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--backend", "mock"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 1, r.stderr[-2000:]
    assert not _json_lines(r.stdout)
    assert "FAILED: exporter ran degraded" in r.stderr, r.stderr[-2000:]


def test_bench_unattributed_single_gpu_fails_loudly():
    env = dict(os.environ, GPUEXP_BENCH_NO_POD_RANK="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--backend", "mock"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 1
    assert not _json_lines(r.stdout)
    assert "FAILED: attributed pods" in r.stderr, r.stderr[-2000:]
