#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): p50 scrape latency + exporter CPU% at N MI355X,
10 Hz, 64 series/GPU, under synthetic HIP-workload pods.

One rank per GPU: under torchrun, or started by this script itself for `--gpus N` > 1
(the parent never touches the GPU).  Rank 0 starts the exporter as a separate process
BEFORE touching the GPU (amdsmi backend, raw gpu_metrics fast path, sentinel kernel on the
aqlprofile PMC queue, full series profile, 10 Hz sampling, every GPU of the job), then
every rank becomes a synthetic "GEMM pod":
each step it launches a burst of bf16 MFMA GEMMs (our HIP kernel) and an RCCL all-reduce
(DP gradient traffic over xGMI; a 1-rank all-reduce at N=1).  The RCCL tracer tool is
injected into every rank, so collective calls/bytes are attributed per pod as well.  Rank 0 scrapes /metrics once per step over a
persistent keep-alive connection with the native client while the GPUs are busy; steps
are paced at the scrape rate.  Each rank's PID is mapped to a fake pod through a pod-map
file, so the per-pod families are exercised too.

value = p50 scrape latency (us, whole job: one exporter serves all N GPUs), lower is
better; exporter CPU% over the timed window is reported alongside.  Scrapes send what
Prometheus sends by default (`Accept-Encoding: gzip`; the exporter compresses once per
tick on the sampler, only while someone asks); latency is request sent -> last response
byte received.  A second timed phase repeats the K steps with identity-encoded (plain
text) responses and reports p50_scrape_identity_us (`--no-gzip` makes that the headline).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "p50 scrape latency + exporter CPU% at 1/2/4/8 MI355X, 10 Hz, 64 series/GPU"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def http_get(port: int, path: str, timeout: float = 2.0) -> tuple[int, bytes]:
    import http.client
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    try:
        c.request("GET", path)
        r = c.getresponse()
        return r.status, r.read()
    finally:
        c.close()


def start_exporter(args, n_gpus: int, backend: str, port: int, pod_map: str, log_path: str, rccl_dir: str = ""):
    cmd = [sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--listen", f"127.0.0.1:{port}",
           "--interval", str(1.0 / args.sample_hz), "--backend", backend,
           "--series-profile", args.series_profile, "--log-level", "warn"]
    if os.environ.get("GPUEXP_BENCH_EXPORTER_ROOT"):
        # an older checkout (A/B hook) may not re-read pod metadata on SIGHUP: poll fast instead
        cmd += ["--control-interval", "0.5"]
    if backend != "mock":
        # Watch exactly the GPUs the ranks run on: HIP device i -> PCI BDF (KFD topology order,
        # read without initialising the GPU), falling back to exporter indices.
        from kubernetes_gpu_exporter_amd.utils.kfdself import hip_order_bdfs
        bdfs = hip_order_bdfs()
        devs = bdfs[:n_gpus] if len(bdfs) >= n_gpus else [str(i) for i in range(n_gpus)]
        cmd += ["--devices", ",".join(devs)]
        if args.sentinel:
            cmd += ["--enable-sentinel", "true"]
        if args.counters:
            cmd += ["--enable-counters", "true"]
        if rccl_dir:
            cmd += ["--enable-rccl", "true", "--rccl-dir", rccl_dir]
    else:
        # Mock devices; the ranks' KFD process entries live in a fake host root that rank 0
        # fills in once it knows every rank's PID (real KFD-reader and attribution path).
        cmd += ["--mock-devices", str(n_gpus), "--enable-sentinel", "true", "--enable-counters", "true",
                "--host-root", args.fake_root]
    if backend == "mock" and getattr(args, "mock_xgmi_file", ""):
        cmd += ["--mock-xgmi-file", args.mock_xgmi_file]
    if getattr(args, "runtime_file", ""):
        cmd += ["--runtime-file", args.runtime_file]
        if args.prewake_ab:  # the A/B's first arm from the start (warm-up included)
            cmd += ["--http-prewake", args.prewake_ab.split(",")[0]]
    env = dict(os.environ)
    env.pop("ROCP_TOOL_LIBRARIES", None)  # the exporter itself issues no collectives
    env["GPUEXP_POD_MAP_FILE"] = pod_map
    env["GPUEXP_POD_ATTRIBUTION"] = "true"
    logf = open(log_path, "a")  # append: a failed first start's output survives the retry
    logf.write(f"--- exporter start {time.strftime('%H:%M:%S')}: {' '.join(cmd)}\n")
    logf.flush()
    if os.environ.get("GPUEXP_BENCH_FAIL_EXPORTER_WITH_COUNTERS") == "1" and args.counters:
        raise RuntimeError("exporter start failed on request (GPUEXP_BENCH_FAIL_EXPORTER_WITH_COUNTERS)")  # test hook
    t_start = time.perf_counter()
    # A/B hook: start the exporter of another checkout (profiles/provenance/tools/devices_ab.sh ran an older
    # round's exporter under this bench's workload); never set in a measurement of this tree
    exp_root = os.environ.get("GPUEXP_BENCH_EXPORTER_ROOT") or ROOT
    proc = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, cwd=exp_root)
    deadline = time.time() + 120
    while time.time() < deadline:
        if proc.poll() is not None:
            raise RuntimeError(f"exporter exited with {proc.returncode}; see {log_path}")
        try:
            st, _ = http_get(port, "/readyz", 0.5)
            if st == 200:
                # process start -> first published sample: amdsmi init + raw-path validation,
                # one HSA queue per GPU (PMC + sentinel), plugin probes, first tick
                proc.startup_s = time.perf_counter() - t_start
                return proc
        except OSError:
            pass
        time.sleep(0.05)
    proc.kill()
    raise RuntimeError("exporter did not become ready")


def pct(v: list, q: float) -> float:
    if not v:
        return float("nan")
    v = sorted(v)
    k = (len(v) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(v) - 1)
    return v[lo] + (v[hi] - v[lo]) * (k - lo)


def startup_budget_s(n_gpus: int) -> float:
    """Exporter start -> first sample: amdsmi + raw-path validation and one HSA queue per GPU.
    Measured on MI355X at 1 GPU: 0.25 s (engine 0.12 s; BENCH_r04.json), so a 20x regression
    fails the run."""
    return 5.0 + 1.5 * n_gpus


def prewake_summary(lat: list, prewoken: list, splits: list) -> dict | None:
    if not lat or len(prewoken) != len(lat):
        return None
    hit = [l for l, p in zip(lat, prewoken) if p == 1]
    miss = [l for l, p in zip(lat, prewoken) if p == 0]
    out = {"timed_scrapes": len(lat), "prewoken": len(hit), "not_prewoken": len(miss),
           "unknown": len(lat) - len(hit) - len(miss),
           "hit_rate": round(len(hit) / len(lat), 3),
           "p50_us_prewoken": round(statistics.median(hit), 2) if hit else None,
           "p50_us_not_prewoken": round(statistics.median(miss), 2) if miss else None}
    for name, flag in (("request_to_server_p50_us_prewoken", 1), ("request_to_server_p50_us_not_prewoken", 0)):
        v = [x[0] for x in splits if x[3] == flag]
        out[name] = round(statistics.median(v), 2) if v else None
    if len(lat) <= 200:  # the driver's short runs: which scrapes, in order (1 pre-woken, 0 not, ? unknown)
        out["sequence"] = "".join("1" if p == 1 else "0" if p == 0 else "?" for p in prewoken)
        out["timed_scrape_us"] = [round(x, 1) for x in lat]
    return out


def request_split(splits: list, q: float) -> dict | None:
    d = [x[4] for x in splits if x[4] is not None]
    w = [x[5] for x in splits if x[5] is not None]
    if not d:
        return None
    return {"send_to_socket_queue": round(pct(d, q), 2), "socket_queue_to_parsed": round(pct(w, q), 2),
            "timestamped": len(d)}


def run_problems(result: dict, n_gpus: int, attribution_ok: bool, rccl_on: bool) -> list:
    """Why a result is not a valid measurement of the configuration, at any N (1 included:
    a run without the PMC counters or the sentinel must not pass for the headline).  Every
    GPU must be exported, every rank's pod attributed, every rank's RCCL communicator span
    all N ranks, no optional source dropped, and the exporter up within its start-up budget."""
    probs = []
    got = len(result["series_per_gpu"])
    if got != n_gpus:
        probs.append(f"series_per_gpu covers {got} GPUs, not {n_gpus}: {sorted(result['series_per_gpu'])}")
    want = {f"gemm-pod-{r}" for r in range(n_gpus)}
    if set(result["attributed_pods"]) != want:
        probs.append(f"attributed pods {result['attributed_pods']} != {sorted(want)}")
    elif not attribution_ok:
        probs.append("attributed pods: not all ranks (or their RCCL communicators) were attributed within the "
                     "untimed 20 s wait before the warm-up")
    if rccl_on:
        ranks = result.get("rccl_rank_per_pod") or {}
        bad = {p: rn for p, rn in ranks.items() if rn[1] != n_gpus}
        missing = sorted(want - set(ranks))
        if bad or missing:
            probs.append(f"RCCL communicators: pods without one {missing}, nranks != {n_gpus}: {bad}")
    reason = result["optional_sources"].get("degraded_reason")
    if reason:
        probs.append(f"exporter ran degraded: {reason}")
    if result["exporter_startup_s"] > result["exporter_startup_budget_s"]:
        probs.append(f"exporter start-up {result['exporter_startup_s']} s > budget {result['exporter_startup_budget_s']} s")
    result["problems"] = probs or None
    return probs


def xgmi_checks(patterns: dict | None, window: dict | None, world: int) -> dict | None:
    """Per-peer sanity of the exporter's xGMI attribution at N > 1 (a SCALE record
    with wrong per-peer attribution must not look as valid as a right one).  Values plus a
    pass flag each; None where the run has no such data (N = 1, pattern phase off):
      cp  every rank's ring_neighbour_share >= 0.9 (a ring uses its two neighbour links);
      ep  every rank's per-peer shares within 20 % of uniform 1 / (N - 1) (all-to-all);
      dp  measured / expected xGMI write of the timed all-reduce within 0.8 .. 1.25."""
    if world <= 1:
        return None
    out: dict = {}
    cp = (patterns or {}).get("cp")
    if cp:
        shares = [r.get("ring_neighbour_share") for r in cp["per_rank"].values()]
        ok = bool(shares) and all(s is not None and s >= 0.9 for s in shares)
        out["cp_ring_neighbour_share_min"] = min((s for s in shares if s is not None), default=None)
        out["cp_ok"] = ok
    ep = (patterns or {}).get("ep")
    if ep:
        uni = 1.0 / (world - 1)
        devs = []
        for r, v in ep["per_rank"].items():
            sh = {p: x for p, x in v.get("per_peer_share", {}).items() if p != r}
            devs.append(max((abs(x / uni - 1.0) for x in sh.values()), default=1.0) if len(sh) == world - 1 else 1.0)
        out["ep_max_deviation_from_uniform"] = round(max(devs), 3) if devs else None
        out["ep_ok"] = bool(devs) and max(devs) <= 0.2
    moe = (window or {}).get("measured_over_expected_write")
    out["dp_measured_over_expected_write"] = moe
    out["dp_ok"] = None if moe is None else 0.8 <= moe <= 1.25
    flags = [v for k, v in out.items() if k.endswith("_ok") and v is not None]
    out["ok"] = all(flags) if flags else None
    return out


def launch_ranks(args, argv: list) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (one per GPU, env
    rendezvous on 127.0.0.1) and relay rank 0's result line.  This parent never imports
    torch or touches a GPU, and never execs: every rank is a child, and the first rank
    that fails takes the others down (their whole process groups, exporter included)."""
    import signal
    port = free_port()
    procs = []
    # rank 0's stdout goes to a file read after every rank exited (a pipe read only then
    # would block rank 0 once it printed more than the pipe buffer)
    out0 = tempfile.TemporaryFile()
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GPUEXP_BENCH_LAUNCHER=str(os.getpid()))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, cwd=ROOT,
                                      stdout=out0 if r == 0 else sys.stderr.fileno(),
                                      start_new_session=True))

    def kill_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def on_signal(signum, _frame):
        kill_all()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    deadline = time.time() + args.launch_timeout
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            break
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and failed is None:
            failed = bad[0]
            print(f"[bench] rank {failed[0]} exited with {failed[1]}; stopping the other ranks", file=sys.stderr,
                  flush=True)
            kill_all()
            grace = time.time() + 20
            while time.time() < grace and any(p.poll() is None for p in procs):
                time.sleep(0.1)
            kill_all(signal.SIGKILL)
        if time.time() > deadline:
            print(f"[bench] ranks still running after {args.launch_timeout} s; stopping them", file=sys.stderr,
                  flush=True)
            kill_all(signal.SIGKILL)
            failed = failed or (-1, 124)
        time.sleep(0.1)
    out0.seek(0)
    out = out0.read().decode(errors="replace")
    out0.close()
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if failed is None and procs[0].returncode == 0 and len(lines) == 1:
        sys.stdout.write(lines[0] + "\n")
        sys.stdout.flush()
        return 0
    if out:
        sys.stderr.write(out)
    rc = procs[0].returncode
    return rc if rc not in (0, None) else (failed[1] if failed and failed[1] > 0 else 1)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--scrape-hz", type=float, default=10.0)
    ap.add_argument("--sample-hz", type=float, default=10.0)
    ap.add_argument("--series-profile", default="full",
                    help="full (default: >= 64 series/GPU incl. counters + reliability) | standard | compact")
    ap.add_argument("--backend", default="auto", help="auto | amdsmi | sysfs | mock")
    ap.add_argument("--gemm", type=int, default=8192, help="GEMM edge (M=N=K) of the synthetic pod")
    ap.add_argument("--busy", type=float, default=0.6, help="target GPU-busy fraction of each step")
    ap.add_argument("--allreduce-mb", type=float, default=64.0)
    ap.add_argument("--gzip", dest="gzip", action="store_true", default=True,
                    help="scrape with Accept-Encoding: gzip, as Prometheus does by default (default)")
    ap.add_argument("--no-gzip", dest="gzip", action="store_false",
                    help="headline scrape with identity encoding (plain text on the wire)")
    ap.add_argument("--identity-phase", type=int, default=1,
                    help="also time K identity-encoded scrapes after the headline phase (p50_scrape_identity_us)")
    ap.add_argument("--proto", action="store_true",
                    help="negotiate the protobuf exposition (Accept: delimited MetricFamily), like Prometheus "
                         "with native histograms")
    ap.add_argument("--sentinel", type=int, default=1)
    ap.add_argument("--counters", type=int, default=1, help="device PMC counters (aqlprofile plugin)")
    ap.add_argument("--out", default="")
    ap.add_argument("--rccl-trace", type=int, default=1,
                    help="inject the RCCL tracer (rocprofiler-sdk tool) into every rank and export per-pod "
                         "collective calls/bytes")
    ap.add_argument("--exporter", choices=("native", "both"), default="native",
                    help="'both' also measures a Python prometheus_client stand-in exporter (utils/refstyle.py)")
    ap.add_argument("--xgmi-patterns", type=int, default=1,
                    help="N > 1: after the timed phases (untimed), drive a ring (CP) and an all-to-all (EP) "
                         "pattern and report each rank's xGMI bytes per peer from the exporter's link counters")
    ap.add_argument("--prewake-ab", default="",
                    help="comma-separated HTTP pre-wake modes (off,slices,spin): the timed scrapes alternate "
                         "between them every --ab-block scrapes inside the one exporter process (switched at "
                         "run time: runtime file + SIGUSR1); per-arm table + block-bootstrap CIs in "
                         "result['prewake_ab'] (utils/abtest.py)")
    ap.add_argument("--ab-block", type=int, default=10, help="timed scrapes per A/B block")
    ap.add_argument("--ab-seed", type=int, default=6, help="seed of the A/B block order")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch (--gpus N > 1 without torchrun): stop the ranks after this many seconds")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)

    # The result line must be the only thing on stdout. RCCL prints its version banner
    # to fd 1 from native code at communicator init, so fd 1 is pointed at stderr for the
    # whole run and the JSON line goes to a private duplicate of the original stdout.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required", file=sys.stderr)
        return 2
    n_gpus = world
    if os.environ.get("GPUEXP_BENCH_FAIL_RANK") == str(rank):  # test hook: a rank that dies at start
        print(f"[bench] rank {rank}: failing on request (GPUEXP_BENCH_FAIL_RANK)", file=sys.stderr)
        return 3

    # RCCL visibility per pod: the tracer tool must be in the environment before the HIP
    # runtime loads (torch's import does that), so set it before importing torch.  All
    # ranks of one launch share the directory the exporter watches.
    rccl_dir = ""
    tracer = os.path.join(ROOT, "kubernetes_gpu_exporter_amd", "libgpuexp_rccl_tracer.so")
    # under rocprofv3 (its preloaded rocprofiler-sdk tool owns the tool slot, so the tracer would
    # never attach and every pod would miss its communicator): no RCCL tracing in that run
    under_rocprof = "rocprofiler-sdk" in os.environ.get("LD_PRELOAD", "") or \
        any(k.startswith("ROCPROF_") for k in os.environ)
    if args.rccl_trace and under_rocprof and rank == 0:
        print("[bench] under rocprofv3: RCCL tracing off for this run", file=sys.stderr, flush=True)
    if args.rccl_trace and not under_rocprof and args.backend != "mock" and os.path.exists(tracer) and \
            os.path.exists("/dev/kfd"):
        # one directory per launch, shared by its ranks (torchrun's static rendezvous names
        # every run "none", so the port tells back-to-back launches apart)
        run_id = "-".join(v for v in (os.environ.get("TORCHELASTIC_RUN_ID"), os.environ.get("MASTER_PORT")) if v) \
            or str(os.getpid())
        rccl_dir = os.path.join(tempfile.gettempdir(), f"gpuexp-bench-rccl-{run_id}")
        os.makedirs(rccl_dir, exist_ok=True)
        os.environ["ROCP_TOOL_LIBRARIES"] = tracer
        os.environ["GPUEXP_RCCL_DIR"] = rccl_dir

    # --- rank 0: exporter first (before this process initialises the GPU) ---
    import torch  # noqa: E402  (import does not initialise HIP; device_count() does not either)
    have_gpu = os.path.exists("/dev/kfd") and torch.cuda.device_count() > 0
    backend = args.backend if args.backend != "auto" else ("amdsmi" if have_gpu else "mock")
    tmpdir = tempfile.mkdtemp(prefix="gpuexp-bench-")
    import atexit
    import shutil
    # (at exit: after the exporter child is stopped; back-to-back launches leave nothing behind)
    atexit.register(shutil.rmtree, tmpdir, True)
    if rank == 0 and os.environ.get("GPUEXP_RCCL_DIR", "").startswith(
            os.path.join(tempfile.gettempdir(), "gpuexp-bench-rccl-")):
        atexit.register(shutil.rmtree, os.environ["GPUEXP_RCCL_DIR"], True)
    pod_map = os.path.join(tmpdir, "podmap.json")
    args.fake_root = os.path.join(tmpdir, "host")
    args.runtime_file = os.path.join(tmpdir, "runtime.yaml") if args.prewake_ab else ""
    # mock backend, N > 1: the ranks' pattern traffic per peer goes into an N x N matrix file
    # the exporter's mock GPUs turn into per-link xGMI bytes (MockBackend::set_traffic_file),
    # so the per-peer checks of the pattern phase run on CPU rehearsals too
    args.mock_xgmi_file = ""
    if backend == "mock" and world > 1:
        run_id = "-".join(v for v in (os.environ.get("TORCHELASTIC_RUN_ID"), os.environ.get("MASTER_PORT")) if v) \
            or str(os.getpid())
        args.mock_xgmi_file = os.path.join(tempfile.gettempdir(), f"gpuexp-bench-xgmi-{run_id}.bin")
        if rank == 0:
            with open(args.mock_xgmi_file, "wb") as fh:
                fh.write(b"\0" * (8 * world * world))
            atexit.register(lambda f=args.mock_xgmi_file: os.path.exists(f) and os.unlink(f))
    mock_sent: dict = {}  # this rank's pattern bytes per peer so far (mock rehearsal)

    def record_mock_traffic(st) -> None:
        if not args.mock_xgmi_file:
            return
        import struct
        for p, b in st.peer_bytes.items():
            mock_sent[p] = mock_sent.get(p, 0) + b
        row = struct.pack(f"<{world}Q", *(int(mock_sent.get(p, 0)) for p in range(world)))
        fd = os.open(args.mock_xgmi_file, os.O_WRONLY)
        try:
            os.pwrite(fd, row, 8 * world * rank)  # this rank's row only: no other writer
        finally:
            os.close(fd)
    os.makedirs(os.path.join(args.fake_root, "sys/class/kfd/kfd/proc"), exist_ok=True)
    port = 0
    exporter = None
    degraded = None
    if rank == 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        port = free_port()
        log_path = os.path.join(ROOT, "gpurun_out", "bench_exporter.log")
        try:
            exporter = start_exporter(args, n_gpus, backend, port, pod_map, log_path, rccl_dir)
        except RuntimeError as ex:
            # Retry without the PMC counters and the sentinel so the run still reports where
            # its time went (--out, stderr), but such a run is degraded: run_problems refuses
            # it, so it exits 1 with no result line, at every N.
            print(f"[bench] exporter start failed ({ex}); retrying without counters/sentinel (the run will be "
                  "reported as degraded, with no result line)", file=sys.stderr, flush=True)
            args.counters, args.sentinel = 0, 0
            degraded = str(ex)
            port = free_port()
            exporter = start_exporter(args, n_gpus, backend, port, pod_map, log_path, rccl_dir)

    dist = None
    if world > 1:
        import torch.distributed as dist
        import datetime
        # a rank that hangs in a collective ends the job in minutes, not after the 10 min default
        dist.init_process_group("nccl" if have_gpu and backend != "mock" else "gloo",  # mock: CPU ranks
                                timeout=datetime.timedelta(seconds=300))
    elif have_gpu and backend != "mock" and args.allreduce_mb > 0:
        # N=1 runs the same data-parallel pod (a 1-rank RCCL all-reduce per step), so the
        # workload and the RCCL path are the same at every N.
        import torch.distributed as dist
        if "MASTER_ADDR" in os.environ:  # torchrun (its agent store serves the rendezvous)
            dist.init_process_group("nccl")
        else:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    use_gpu = have_gpu and backend != "mock"
    if use_gpu:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:
        dev = torch.device("cpu")

    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.k8s.filesource import write_pod_map
    from kubernetes_gpu_exporter_amd.utils import promproto, promtext
    from kubernetes_gpu_exporter_amd.utils.fakehost import FakeHost, kubepods_cgroup
    from kubernetes_gpu_exporter_amd.utils.procstat import cpu_seconds_precise, thread_cpu_ns_by_name
    n = load()
    from kubernetes_gpu_exporter_amd.ops.gemm import kernels
    kern = kernels() if use_gpu else None

    # --- synthetic GEMM pod workload ---
    G = args.gemm
    stream = 0
    if use_gpu:
        a = torch.empty(G, G, device=dev, dtype=torch.bfloat16)
        b = torch.empty(G, G, device=dev, dtype=torch.bfloat16)
        c = torch.empty(G, G, device=dev, dtype=torch.bfloat16)
        stream = torch.cuda.current_stream().cuda_stream
        kern.fill_bf16(a.data_ptr(), a.numel(), 1 + rank, stream)
        kern.fill_bf16(b.data_ptr(), b.numel(), 7 + rank, stream)
        grad = torch.ones(int(args.allreduce_mb * (1 << 20)) // 2, device=dev, dtype=torch.bfloat16)
    else:
        grad = torch.ones(1024)

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    def gemm_burst(iters: int):
        for _ in range(iters):
            kern.gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), G, G, G, stream)

    period = 1.0 / args.scrape_hz
    iters = 0
    gemm_ms = 0.0
    if use_gpu:
        # GEMM time from GPU events over 20 back-to-back dispatches after a 10-dispatch
        # warm-up (clocks settled): the rate rocprofv3's kernel trace gives, not a host timer
        # around a handful of launches
        gemm_burst(10)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        gemm_burst(20)
        ev1.record()
        sync()
        gemm_ms = ev0.elapsed_time(ev1) / 20
        iters = max(1, int(args.busy * period * 1e3 / gemm_ms))
        if dist is not None:
            t = torch.tensor([iters], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            iters = int(t.item())

    # --- pod map: every rank's PID -> fake pod bench/gemm-pod-<rank> ---
    own_pid = pid = os.getpid()
    if use_gpu:
        # KFD names processes by HOST pid; inside a PID namespace (no hostPID) find ours by
        # a VRAM fingerprint so the exporter can attribute this rank to its fake pod.
        from kubernetes_gpu_exporter_amd.utils.kfdself import find_own_kfd_pid
        pid = find_own_kfd_pid(local_rank, salt=rank) or pid
    my_bdf = ""
    if use_gpu:
        from kubernetes_gpu_exporter_amd.utils.kfdself import hip_order_bdfs
        order = hip_order_bdfs()
        my_bdf = order[local_rank].lower() if local_rank < len(order) else ""
    elif backend == "mock":
        my_bdf = f"0000:{0x10 + 0x10 * rank:02x}:00.0"  # mock GPU `rank` (backend_mock.cc)
    if dist is not None:
        pids = [None] * world
        dist.all_gather_object(pids, (pid, own_pid, my_bdf))
    else:
        pids = [(pid, own_pid, my_bdf)]
    attribution_ok = True
    if rank == 0:
        pods, cgroups = [], {}
        hidden = os.environ.get("GPUEXP_BENCH_NO_POD_RANK")  # test hook: this rank's pod never attributes
        for r, (p, op, _) in enumerate(pids):
            if hidden == str(r):
                continue
            uid = f"00000000-0000-4000-8000-{r:012d}"
            cid = f"{r:064x}"
            pods.append({"uid": uid, "namespace": "bench", "name": f"gemm-pod-{r}", "containers": {cid: "worker"}})
            # KFD names the rank by host PID; the RCCL tracer by its PID in the exporter's
            # namespace — the same number unless the box runs us in a PID namespace
            cgroups[p] = cgroups[op] = kubepods_cgroup(uid, cid, qos="guaranteed")
            if not use_gpu:
                # mock GPU r (KFD gpu_id 1000 + r) holds rank r's buffers
                FakeHost(args.fake_root).set_process_gpu(p, 1000 + r, vram=(r + 1) << 30, cu=32)
        write_pod_map(pod_map, pods, cgroups)
        if exporter is not None and not os.environ.get("GPUEXP_BENCH_EXPORTER_ROOT"):
            # the exporter's control plane refreshes every 5 s (its default); SIGHUP makes it
            # read the new pod map now
            exporter.send_signal(signal.SIGHUP)
        # Untimed: wait until the exporter has picked the pod map up and attributes every
        # rank (SIGHUP above: its control plane re-reads the file at once), so even a short warmup
        # measures the steady state.
        # With the RCCL tracer on, also until every rank's communicator is attributed to its
        # pod (each rank has run collectives by now: the GEMM-count all-reduce above).
        want = {p["name"] for p in pods}
        t_attr = time.time() + 20
        while time.time() < t_attr:
            try:
                st, body = http_get(port, "/metrics", 2.0)
                fams0 = promtext.parse(body.decode())
                got = {lab["pod"] for _, lab, _ in promtext.samples(fams0, "pod_gpu_memory_usage")}
                comm = {lab["pod"] for _, lab, _ in promtext.samples(fams0, "amd_rccl_communicator_info")}
                if st == 200 and want <= got and (not rccl_dir or want <= comm):
                    break
            except OSError:
                pass
            time.sleep(0.1)
        else:
            attribution_ok = False
            print(f"[bench] exporter did not attribute all {len(want)} ranks (GPU processes"
                  f"{' and RCCL communicators' if rccl_dir else ''}) within 20 s", file=sys.stderr, flush=True)
        # timing=True: the server echoes when it parsed the request and started writing,
        # so each latency splits into request wake-up / server work / response delivery
        client = n.ScrapeClient("127.0.0.1", port, "/metrics", args.gzip, 5000,
                                promproto.ACCEPT if args.proto else "", True)
    else:
        client = None

    splits: list = []
    prewoken: list = []  # per timed headline scrape: 1 pre-woken worker, 0 not, -1 unknown
    # --prewake-ab: the arm of each block of timed scrapes, the blocks measured so far, and the
    # arm to switch the exporter to right after the next scrape (its ~100 ms idle gap follows)
    from kubernetes_gpu_exporter_amd.utils import abtest
    ab_arms = [a.strip() for a in args.prewake_ab.split(",") if a.strip()]
    ab_blocks: list = []
    ab_state = {"next": None, "cur": None, "t0": 0.0, "http0": 0, "proc0": 0}

    def ab_boundary():
        """Closes the current A/B block (wall and CPU since it began) and switches the
        exporter to ab_state['next'] (runtime file + SIGUSR1)."""
        th = thread_cpu_ns_by_name(exporter.pid)
        now = time.perf_counter()
        http_ns, proc_ns = sum(v for k, v in th.items() if k.startswith("gpuexp-http")), sum(th.values())
        if ab_state["cur"] is not None and ab_blocks:
            b = ab_blocks[-1]
            b.wall_s, b.http_cpu_ns, b.proc_cpu_ns = now - ab_state["t0"], http_ns - ab_state["http0"], \
                proc_ns - ab_state["proc0"]
        nxt = ab_state["next"]
        ab_state.update(next=None, cur=nxt, t0=now, http0=http_ns, proc0=proc_ns)
        if nxt is not None:
            with open(args.runtime_file, "w") as fh:
                fh.write(f"http_prewake: {nxt}\n")
            exporter.send_signal(signal.SIGUSR1)
            ab_blocks.append(abtest.Block(nxt))
            if len(ab_blocks) % 10 == 1:  # progress (a long A/B must not look hung)
                print(f"[bench] A/B block {len(ab_blocks)}/{len(ab_sched)}: {nxt}", file=sys.stderr, flush=True)

    def step(cl, lat: list | None, after_scrape=None):
        t_start = time.perf_counter()
        if use_gpu:
            gemm_burst(iters)
        if rank == 0:
            ns = cl.scrape()  # GPUs are busy with the burst while we scrape
            if lat is not None and ns >= 0:
                lat.append(ns / 1e3)
                if cl is client:
                    t_send, t_parse, t_write, t_done = cl.last_timing()
                    pw = cl.last_prewoken()
                    rx = cl.last_server_rx()  # kernel receive time of the request on the server socket
                    prewoken.append(pw)
                    rec = {"total": ns / 1e3, "pw": pw}
                    if t_parse and t_send <= t_parse <= t_write <= t_done:
                        rx_ok = bool(rx) and t_send <= rx <= t_parse
                        splits.append(((t_parse - t_send) / 1e3, (t_write - t_parse) / 1e3, (t_done - t_write) / 1e3,
                                       pw, (rx - t_send) / 1e3 if rx_ok else None,
                                       (t_parse - rx) / 1e3 if rx_ok else None))
                        rec["req"] = (t_parse - t_send) / 1e3
                        rec["sq"] = (t_parse - rx) / 1e3 if rx_ok else None
                    if ab_arms and ab_blocks and ab_state["cur"] is not None:
                        ab_blocks[-1].scrapes.append(rec)
            if ab_arms and cl is client and (ab_state["next"] is not None or ab_state["cur"] is not None):
                if ab_state["next"] is not None or (ab_blocks and len(ab_blocks[-1].scrapes) >= args.ab_block):
                    if ab_state["next"] is None:  # block full: the next arm of the schedule
                        ab_state["next"] = ab_sched[len(ab_blocks)] if len(ab_blocks) < len(ab_sched) else None
                    ab_boundary()
            if after_scrape is not None:
                after_scrape()
        if dist is not None:
            dist.all_reduce(grad)
        sync()
        rest = period - (time.perf_counter() - t_start)
        if rest > 0:
            time.sleep(rest)

    def last_fams(cl):
        body = cl.last_body()
        if args.gzip:
            body = __import__("gzip").decompress(body)
        return promtext.parse(body.decode()) if body[:1] == b"#" else \
            promproto.to_promtext(promproto.parse_delimited(body))

    def xgmi_totals(cl) -> tuple[float, dict]:
        """(time, {gpu: [read_bytes, write_bytes]}) summed over links, from the exporter's
        hardware-accumulator counters in the body of the scrape `cl` just did."""
        fams = last_fams(cl)
        tot: dict = {}
        for k, fam_name in enumerate(("amd_gpu_xgmi_read_bytes_total", "amd_gpu_xgmi_write_bytes_total")):
            for _, lab, v in promtext.samples(fams, fam_name):
                tot.setdefault(lab.get("gpu"), [0.0, 0.0])[k] += v
        return time.perf_counter(), tot

    def xgmi_links(cl) -> dict:
        """{(bdf, peer_bdf): [read_bytes, write_bytes]} per xGMI link, from a fresh scrape
        ({} if the scrape fails: rank 0 must still reach every collective of the phase)."""
        out: dict = {}
        try:
            if cl.scrape() < 0:
                return out
            fams = last_fams(cl)
        except Exception as ex:  # noqa: BLE001
            print(f"[bench] xgmi pattern scrape failed: {ex}", file=sys.stderr, flush=True)
            return out
        for k, fam_name in enumerate(("amd_gpu_xgmi_read_bytes_total", "amd_gpu_xgmi_write_bytes_total")):
            for _, lab, v in promtext.samples(fams, fam_name):
                key = (lab.get("bdf", "").lower(), lab.get("peer_bdf", "").lower())
                out.setdefault(key, [0.0, 0.0])[k] += v
        return out

    def xgmi_patterns(cl, bdfs: list) -> dict:
        """Untimed, after the measured phases (N > 1 only): drives two traffic patterns with
        known peers and reports, per rank, where its xGMI bytes went according to the
        exporter's per-link accumulators (peer_bdf labels):
          cp  ring (context parallel): rank r sends to r+1 and receives from r-1, so its
              link bytes should sit on the links to its two ring neighbours;
          ep  all-to-all (expert parallel): every peer gets an equal share.
        `bdfs[r]` is rank r's GPU.  Returns {pattern: {...}}; the share values are what the
        per-peer attribution must get right."""
        from kubernetes_gpu_exporter_amd.parallel.collectives import run as run_pattern
        out: dict = {}
        nb, target_s = (256 << 20, 1.0) if use_gpu else (4 << 20, 0.2)  # mock: gloo on the CPU
        for pattern in ("cp", "ep"):
            # check=False throughout: a rank that raised here would leave the others in a
            # collective (the generators' results are verified by the tests instead)
            record_mock_traffic(run_pattern(pattern, steps=1, nbytes=nb, device=dev, check=False))  # warm-up
            sync()
            t = time.perf_counter()
            record_mock_traffic(run_pattern(pattern, steps=1, nbytes=nb, device=dev, check=False))
            sync()
            steps = torch.tensor([max(1, int(target_s / max(1e-4, time.perf_counter() - t)))], device=dev)
            dist.all_reduce(steps, op=dist.ReduceOp.MAX)  # every rank runs the same step count
            dist.barrier()
            before = None
            if rank == 0:
                time.sleep(0.3)  # idle: the accumulators of the last tick are final
                before = xgmi_links(cl)
            dist.barrier()
            t0 = time.perf_counter()
            st = run_pattern(pattern, steps=int(steps.item()), nbytes=nb, device=dev, check=False)
            sync()
            record_mock_traffic(st)
            dist.barrier()
            if rank != 0:
                continue
            secs = time.perf_counter() - t0
            time.sleep(0.3)  # two sample ticks: the window's last bytes are in the accumulators
            after = xgmi_links(cl)
            per_rank = {}
            for r, b in enumerate(bdfs):
                peers, rw = {}, [0.0, 0.0]
                for (src, peer), v in after.items():
                    if src != b:
                        continue
                    v0 = before.get((src, peer), [0.0, 0.0])
                    d = [v[0] - v0[0], v[1] - v0[1]]
                    rw = [rw[0] + d[0], rw[1] + d[1]]
                    pr = str(bdfs.index(peer)) if peer in bdfs else (peer or "?")
                    peers[pr] = peers.get(pr, 0.0) + d[0] + d[1]
                total = sum(peers.values())
                entry = {"read_bytes": round(rw[0]), "write_bytes": round(rw[1]),
                         "per_peer_share": {k: round(v / total, 3) for k, v in sorted(peers.items()) if total}}
                if pattern == "cp" and total:
                    nbr = {str((r + 1) % world), str((r - 1) % world)}
                    entry["ring_neighbour_share"] = round(sum(v for k, v in peers.items() if k in nbr) / total, 3)
                per_rank[str(r)] = entry
            sent = sum(st.bytes.values()) / 2 if pattern == "cp" else st.bytes.get("alltoall", 0) * (world - 1) / world
            out[pattern] = {"steps": int(steps.item()), "seconds": round(secs, 3),
                            "expected_bytes_out_per_rank": round(sent), "per_rank": per_rank}
        return out

    xgmi_window: dict = {}
    fresh0: dict = {}  # per-GPU fresh gpu_metrics reads at the start of the timed window
    counters0: dict = {}  # exporter self counters at the start of the timed window
    expo0: dict = {}  # compiled-exposition events (relayouts, ...) and ticks at the window's start
    window_s = [0.0]

    stage0: dict = {}  # per-stage (sum, count) of the tick-time histogram at the window's start

    def stage_sums(fams) -> dict:
        out: dict = {}
        for sname, lab, v in fams.get("gpuexp_sample_stage_duration_seconds", promtext.Family("x")).samples:
            if sname.endswith("_sum"):
                out.setdefault(lab["stage"], [0.0, 0.0])[0] = v
            elif sname.endswith("_count"):
                out.setdefault(lab["stage"], [0.0, 0.0])[1] = v
        return out

    def fresh_reads(fams) -> dict:
        return {lab["gpu"]: v for _, lab, v in promtext.samples(fams, "gpuexp_gpu_metrics_reads_total")
                if lab.get("kind") == "fresh"}
    exporter_rss_kb = [0]
    cpu_by_thread: dict = {}

    def phase(proc, cl, native_exporter: bool = False):
        """W untimed + K timed steps (barrier + synchronize on both sides); returns the
        latencies, exporter CPU% over the timed window and max-over-ranks ms/step."""
        x0 = None

        def window_start():
            """xGMI accumulators and self counters at the start of the window (untimed), on a
            connection of its own: an extra request on the timed connection would break the
            steady scrape period the server learns per connection (pre-wake), as Prometheus
            never does.  Runs inside the last warm-up step, right after its scrape, so its
            time comes out of that step's idle rest: run between the steps it made the first
            timed scrape late by the side scrape + parse, past the pre-wake window
            (profiles/r06/session4: "0111...")."""
            nonlocal x0
            side = n.ScrapeClient("127.0.0.1", port, "/metrics", args.gzip, 5000,
                                  promproto.ACCEPT if args.proto else "")
            side.scrape()
            x0 = xgmi_totals(side)
            f0 = last_fams(side)
            fresh0.clear()
            fresh0.update(fresh_reads(f0))
            stage0.clear()
            stage0.update(stage_sums(f0))
            expo0.clear()
            expo0.update({lab.get("event"): v for _, lab, v in promtext.samples(f0, "gpuexp_exposition_events_total")})
            expo0.update({"ticks": v for _, _, v in promtext.samples(f0, "gpuexp_ticks_total")})
            for name in ("gpuexp_http_prewake_hits_total", "gpuexp_http_prewake_hits_narrow_total",
                         "gpuexp_scrapes_total"):
                v = [x for _, _, x in promtext.samples(f0, name)]
                if v:
                    counters0[name] = v[0]

        capture = native_exporter and rank == 0  # (mock backends too: the CPU tests run this path)
        for w in range(args.warmup):
            if ab_arms and native_exporter and rank == 0 and w == args.warmup - 1:
                ab_state["next"] = ab_sched[0]  # the first block's arm, switched after this scrape
            step(cl, None, window_start if capture and w == args.warmup - 1 else None)
        if capture and x0 is None:  # no warm-up
            window_start()
        if dist is not None:
            dist.barrier()
        sync()
        lat: list = []
        cpu0 = cpu_seconds_precise(proc.pid) if rank == 0 else 0.0
        by0 = thread_cpu_ns_by_name(proc.pid) if rank == 0 else {}
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(cl, lat)
        if dist is not None:
            dist.barrier()
        sync()
        elapsed = time.perf_counter() - t0
        if native_exporter:
            window_s[0] = elapsed
        cpu_pct = 100.0 * (cpu_seconds_precise(proc.pid) - cpu0) / elapsed if rank == 0 else 0.0
        if rank == 0 and native_exporter:
            # where the exporter's CPU went, per thread name (us per step over the window)
            by1 = thread_cpu_ns_by_name(proc.pid)
            cpu_by_thread.clear()
            cpu_by_thread.update({k: round((v - by0.get(k, 0)) / 1e3 / max(1, args.steps), 1)
                                  for k, v in sorted(by1.items()) if v - by0.get(k, 0) > 0})
            try:  # resident memory of the exporter: each GPU queue it holds pins a CWSR area
                exporter_rss_kb[0] = int([l for l in open(f"/proc/{proc.pid}/status")
                                          if l.startswith("VmRSS:")][0].split()[1])
            except (OSError, IndexError, ValueError):
                pass
        if x0 is not None and use_gpu:  # (mock links carry no all-reduce bytes)
            # xGMI bytes the hardware counted over the window vs what the DP all-reduce must
            # move: 2(N-1)/N x buffer per GPU per step for any bandwidth-optimal algorithm
            # (ring or direct); counters lag by <= one sample period (100 ms at 10 Hz).
            t1, tot1 = xgmi_totals(cl)
            dt = t1 - x0[0]
            per_gpu = {g: {"read_Bps": round((v[0] - x0[1].get(g, [0, 0])[0]) / dt),
                           "write_Bps": round((v[1] - x0[1].get(g, [0, 0])[1]) / dt)} for g, v in tot1.items()}
            buf = grad.numel() * grad.element_size()
            expect = 2.0 * (world - 1) / world * buf * args.steps / elapsed if dist is not None else 0.0
            xgmi_window.update({"window_s": round(dt, 3), "per_gpu": per_gpu,
                                "expected_allreduce_Bps_per_gpu": round(expect)})
            if expect > 0 and per_gpu:
                xgmi_window["measured_over_expected_write"] = round(
                    statistics.mean(v["write_Bps"] for v in per_gpu.values()) / expect, 3)
        msps = elapsed / max(1, args.steps) * 1e3
        if dist is not None:
            t = torch.tensor([msps], device=dev if use_gpu else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            msps = float(t.item())
        return lat, cpu_pct, msps

    def stop_proc(proc):
        proc.terminate()
        try:
            proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()

    ab_sched = abtest.block_schedule(ab_arms, (args.steps + args.ab_block - 1) // args.ab_block, args.ab_seed) \
        if ab_arms else []
    if ab_arms and args.warmup < 1:
        print("[bench] --prewake-ab needs --warmup >= 1 (the first arm is switched after the last warm-up scrape)",
              file=sys.stderr)
        return 2
    lat, cpu_pct, ms_per_step = phase(exporter, client if rank == 0 else None, native_exporter=True)
    if ab_arms and rank == 0 and ab_state["cur"] is not None:
        ab_boundary()  # closes the last block
    lat_id = cpu_id = None
    if args.identity_phase and args.gzip and not ab_arms:
        # Same workload, same exporter, plain-text (identity) responses: the bytes on the
        # wire grow with the GPU count here, gzip'd ones barely do.
        id_client = n.ScrapeClient("127.0.0.1", port, "/metrics", False, 5000,
                                   promproto.ACCEPT if args.proto else "") if rank == 0 else None
        lat_id, cpu_id, _ = phase(exporter, id_client)
        if rank == 0:
            id_bytes = id_client.last_bytes

    result = None
    if rank == 0:
        body = client.last_body()
        if args.gzip:
            body = __import__("gzip").decompress(body)
        if os.environ.get("GPUEXP_BENCH_DUMP_EXPOSITION"):  # evidence: the last timed scrape's body
            with open(os.environ["GPUEXP_BENCH_DUMP_EXPOSITION"], "wb") as f:
                f.write(body)
        if body[:1] == b"#":
            fams = promtext.parse(body.decode())
        else:  # protobuf exposition
            fams = promproto.to_promtext(promproto.parse_delimited(body))
        per_gpu: dict = {}
        for name, fam in fams.items():
            if name.startswith("amd_gpu_") and not name.startswith("amd_gpu_process_"):
                for _, lab, _ in fam.samples:
                    per_gpu[lab.get("gpu")] = per_gpu.get(lab.get("gpu"), 0) + 1
        attributed = {lab["pod"] for _, lab, _ in fams.get("pod_gpu_memory_usage", promtext.Family("x")).samples}
        sentinel = {}
        for key, fam_name in (("sclk_hz", "amd_gpu_sentinel_sclk_hz"),
                              ("dispatch_latency_s", "amd_gpu_sentinel_dispatch_latency_seconds")):
            v = [s[2] for s in promtext.samples(fams, fam_name)]
            if v:
                sentinel[key] = statistics.median(v)
        gfx = [s[2] for s in promtext.samples(fams, "amd_gpu_gfx_activity_percent")]
        # diagnostics: which device families GPU 0 exports, and where the sampler's time goes
        fam_gpu0 = {name: sum(1 for _, lab, _ in fam.samples if lab.get("gpu") == "0")
                    for name, fam in fams.items() if name.startswith("amd_gpu_")
                    and not name.startswith("amd_gpu_process_")}
        stage_raw = stage_sums(fams)
        stage_us = {k: round(a / c * 1e6, 2) for k, (a, c) in stage_raw.items() if c}
        # the same between the histogram publications around the timed window (published at most
        # once a second; sum and count come from the same publication): start-up's first renders
        # (every family laid out) dominate a short run's whole-run mean
        stage_us_window = {k: round((a - stage0[k][0]) / (c - stage0[k][1]) * 1e6, 2)
                           for k, (a, c) in stage_raw.items()
                           if k in stage0 and stage0[k][1] > 0 and c > stage0[k][1]} or None  # (None: not
        # published before the window -- a warm-up under a second)
        # p50 per stage from the cumulative histogram buckets (upper bound of the median bucket)
        buckets: dict = {}
        for sname, lab, v in fams.get("gpuexp_sample_stage_duration_seconds", promtext.Family("x")).samples:
            if sname.endswith("_bucket"):
                buckets.setdefault(lab["stage"], []).append((float(lab["le"]), v))  # "+Inf" -> inf
        stage_p50_us = {}
        for st_name, bl in buckets.items():
            bl.sort()
            total = bl[-1][1]
            le50 = next((le for le, v in bl if total and v >= total / 2), None)
            stage_p50_us[st_name] = round(le50 * 1e6, 1) if le50 is not None else None
        # server side of a scrape (request parsed -> last byte written), all scrapes so far:
        # the rest of the client-measured latency is loopback TCP + thread wake-ups
        srv = {s[0].rsplit("_", 1)[-1]: s[2] for s in promtext.samples(fams, "gpuexp_scrape_duration_seconds")
               if s[0].endswith(("_sum", "_count"))}
        server_mean_us = round(srv["sum"] / srv["count"] * 1e6, 2) if srv.get("count") else None
        # server-side p50/p99 over EVERY scrape of the run (warmup, both phases): upper
        # bound of the histogram bucket holding the quantile
        sb = sorted((float(lab["le"]), v) for _, lab, v in promtext.samples(fams, "gpuexp_scrape_duration_seconds")
                    if "le" in lab)
        server_q = {}
        if sb and sb[-1][1]:
            for qname, q in (("p50", 0.5), ("p99", 0.99)):
                le = next(le for le, v in sb if v >= q * sb[-1][1])
                server_q[qname] = round(le * 1e6, 1) if le != float("inf") else None
        server_scrapes = int(sb[-1][1]) if sb else 0
        ticks = [v for _, _, v in promtext.samples(fams, "gpuexp_ticks_total")]
        metrics_reads = {lab["kind"]: v for _, lab, v in promtext.samples(fams, "gpuexp_gpu_metrics_reads_total")
                         if lab.get("gpu") == "0"}
        sampler_cpu = [v for _, _, v in promtext.samples(fams, "gpuexp_sampler_cpu_seconds_total")]
        # the devices stage split (whole run): mean per tick of each part, summed over GPUs
        dev_parts = {lab["part"]: v for _, lab, v in promtext.samples(fams, "gpuexp_device_read_seconds_total")}
        fetch_cpu = {lab["gpu"]: v for _, lab, v in promtext.samples(fams, "gpuexp_gpu_metrics_fetch_cpu_seconds_total")}
        fetch_cap = {lab["gpu"]: v for _, lab, v in promtext.samples(fams, "gpuexp_gpu_metrics_min_interval_seconds")}
        prewake = [v for _, _, v in promtext.samples(fams, "gpuexp_http_prewake_wakeups_total")]
        scrapes_total = [v for _, _, v in promtext.samples(fams, "gpuexp_scrapes_total")]
        gz_where = {lab.get("where"): int(v) for _, lab, v in promtext.samples(fams, "gpuexp_gzip_compressions_total")}
        # render_when_due: ticks that rendered nothing because no steady scraper was due (whole run)
        expo_events = {lab.get("event"): int(v) for _, lab, v in promtext.samples(fams, "gpuexp_exposition_events_total")}
        rccl = {}
        for sname, lab, v in promtext.samples(fams, "amd_rccl_collective_bytes_total"):
            rccl.setdefault(lab.get("pod") or lab.get("pid"), {}).setdefault(lab["op"], {})["bytes"] = v
        for sname, lab, v in promtext.samples(fams, "amd_rccl_collective_calls_total"):
            rccl.setdefault(lab.get("pod") or lab.get("pid"), {}).setdefault(lab["op"], {})["calls"] = v
        rccl_files = {lab.get("state"): int(v) for _, lab, v in promtext.samples(fams, "gpuexp_rccl_files")}
        rccl_ranks = {lab.get("pod") or lab.get("pid"): [int(lab["rank"]), int(lab["nranks"])]
                      for _, lab, _ in promtext.samples(fams, "amd_rccl_communicator_info")}
        xgmi = {}
        for fam_name, key in (("amd_gpu_xgmi_read_bytes_per_second", "read"),
                              ("amd_gpu_xgmi_write_bytes_per_second", "write")):
            for _, lab, v in promtext.samples(fams, fam_name):
                xgmi.setdefault(lab.get("gpu"), {})[key] = v
        tflops = 2.0 * G ** 3 * iters / (gemm_ms * iters * 1e-3) / 1e12 if gemm_ms else None
        # how often each GPU's gpu_metrics table was fetched fresh over the timed window (the
        # auto fetch policy caps it at 1 / gpuexp_gpu_metrics_min_interval_seconds: at 8 GPUs a
        # "10 Hz" exporter refreshes power / clocks / activity at ~3-5 Hz)
        fresh1 = fresh_reads(fams)
        fresh_hz = ({g: round((fresh1[g] - fresh0[g]) / window_s[0], 2) for g in sorted(fresh1, key=int)
                     if g in fresh0} if fresh0 and window_s[0] > 0 else None)
        result = {
            "metric": METRIC,
            "value": round(statistics.median(lat), 2) if lat else None,
            "unit": "us",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": f"mi355x-per-pod-exporter ({args.series_profile} profile) + bf16 MFMA GEMM pods",
                       "global_batch": n_gpus, "seq_len": 0, "parallelism": f"dp{n_gpus}",
                       "scrape_hz": args.scrape_hz, "sample_hz": args.sample_hz, "backend": backend,
                       "series_profile": args.series_profile, "gzip": args.gzip, "protobuf": args.proto,
                       "gemm": f"{G}^3 x {iters}/step",
                       "gemm_kernel_variant": kern.gemm_variant(G, G, G, 0) if kern is not None else None,
                       "allreduce_mb": args.allreduce_mb if dist is not None else 0,
                       "gpu_metrics_fresh_hz": fresh_hz},
            "p50_scrape_us": round(statistics.median(lat), 2) if lat else None,
            # a p99 needs >= 100 samples; below that only the max of the timed scrapes and
            # the server-side histogram quantiles over every scrape of the run are given
            "p99_scrape_us": round(pct(lat, 0.99), 2) if len(lat) >= 100 else None,
            "max_scrape_us": round(max(lat), 2) if lat else None,
            "server_scrape_p50_le_us": server_q.get("p50"),
            "server_scrape_p99_le_us": server_q.get("p99"),
            "server_scrapes": server_scrapes,
            "exporter_cpu_percent": round(cpu_pct, 3),
            "exporter_cpu_us_per_step_by_thread": cpu_by_thread,
            "exporter_rss_mb": round(exporter_rss_kb[0] / 1024, 1) if exporter_rss_kb[0] else None,
            "exporter_startup_s": round(getattr(exporter, "startup_s", 0.0), 2),
            # the engine's own share of it (start() -> first sample; gpuexp_startup_seconds)
            "engine_startup_s": next((round(v, 3) for _, _, v in promtext.samples(fams, "gpuexp_startup_seconds")),
                                     None),
            "exporter_startup_budget_s": startup_budget_s(n_gpus),
            "scrape_encoding": "gzip (Prometheus default Accept-Encoding)" if args.gzip else "identity",
            "p50_scrape_identity_us": round(statistics.median(lat_id), 2) if lat_id else None,
            "p99_scrape_identity_us": round(pct(lat_id, 0.99), 2) if lat_id and len(lat_id) >= 100 else None,
            "exporter_cpu_percent_identity_phase": round(cpu_id, 3) if cpu_id is not None else None,
            "scrape_bytes_identity": id_bytes if lat_id else None,
            "server_scrape_mean_us": server_mean_us,
            # per-scrape split (medians of each part; same-host CLOCK_MONOTONIC): request sent ->
            # server parsed it (loopback + server thread wake-up), server parse -> write start,
            # write start -> client has the last byte (copy + client wake-up)
            "latency_split_p50_us": {
                "request_to_server": round(statistics.median(x[0] for x in splits), 2),
                "server_work": round(statistics.median(x[1] for x in splits), 2),
                "response_to_client": round(statistics.median(x[2] for x in splits), 2)} if splits else None,
            "latency_split_p90_us": {
                "request_to_server": round(pct([x[0] for x in splits], 0.9), 2),
                "server_work": round(pct([x[1] for x in splits], 0.9), 2),
                "response_to_client": round(pct([x[2] for x in splits], 0.9), 2)} if splits else None,
            # request_to_server split by the kernel's receive timestamp on the server socket:
            # client send() -> request queued on the server socket (loopback delivery), and
            # queued -> parsed (the server thread's wake-up + read)
            "request_split_p50_us": request_split(splits, 0.5),
            "request_split_p90_us": request_split(splits, 0.9),
            # every timed scrape accounted for: did it reach an HTTP worker that its pre-wake
            # timer had already woken (gpuexp_http_prewake_hits_total), or one asleep in epoll?
            "prewake": prewake_summary(lat, prewoken, splits),
            # scrapes of the timed window (+ the window-start side scrape) pre-woken under the current
            # hit window (lead + jitter allowance + one slice) and under round 3's (lead + one slice)
            "prewake_hits_window": {
                k: round(next((x for _, _, x in promtext.samples(fams, name)), 0.0) - counters0[name])
                for k, name in (("hits", "gpuexp_http_prewake_hits_total"),
                                ("hits_round3_window", "gpuexp_http_prewake_hits_narrow_total"),
                                ("scrapes", "gpuexp_scrapes_total")) if name in counters0} or None,
            # exporter settings the run overrode through the environment (A/B arms)
            "exporter_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("GPUEXP_")
                             and k not in ("GPUEXP_BENCH_DUMP_EXPOSITION",)} or None,
            "scrapes": len(lat),
            "scrape_errors": client.errors,
            "scrape_bytes": client.last_bytes,
            "series_per_gpu": dict(sorted((k, v) for k, v in per_gpu.items() if k is not None)),
            "attributed_pods": sorted(attributed),
            "gpu_gfx_activity_percent": gfx,
            "sentinel": sentinel,
            "workload_gemm_tflops_per_gpu": round(tflops, 1) if tflops else None,
            "rccl_per_pod": rccl,
            "rccl_rank_per_pod": rccl_ranks,
            "rccl_files": rccl_files or None,  # tracer files by state (active = writer proven)
            "xgmi_bytes_per_second": xgmi,
            # xGMI bytes the exporter's hardware counters saw vs what the DP all-reduce had to
            # move (null at 1 rank: nothing crosses xGMI; null on the mock backend)
            "xgmi_timed_window": dict({"measured_over_expected_write": None}, **xgmi_window),
            "families_gpu0": {k: v for k, v in sorted(fam_gpu0.items()) if v},
            "sample_stage_mean_us": stage_us,
            "sample_stage_mean_us_timed_window": stage_us_window,
            "sample_stage_p50_le_us": stage_p50_us,
            "gpu_metrics_reads_gpu0": metrics_reads,
            "device_read_mean_us_per_tick": {k: round(v / ticks[0] * 1e6, 2) for k, v in sorted(dev_parts.items())}
            if dev_parts and ticks and ticks[0] else None,
            "gpu_metrics_fetch_cpu_us_per_fresh_read_gpu0": round(fetch_cpu["0"] / metrics_reads["fresh"] * 1e6, 1)
            if fetch_cpu.get("0") and metrics_reads.get("fresh") else None,
            "gpu_metrics_min_interval_s": fetch_cap or None,
            "gpu_metrics_fresh_hz": fresh_hz,
            "counters_kick": os.environ.get("GPUEXP_COUNTERS_KICK", "default"),
            "sampler_thread_cpu_s": sampler_cpu[0] if sampler_cpu else None,
            "sampler_cpu_us_per_tick": round(sampler_cpu[0] / ticks[0] * 1e6, 1) if sampler_cpu and ticks and ticks[0]
            else None,
            "sampler_cpu_us_per_tick_per_gpu": round(sampler_cpu[0] / ticks[0] * 1e6 / n_gpus, 1)
            if sampler_cpu and ticks and ticks[0] else None,
            "ranks": world,
            # gzip copies made by the sampler (scrape expected before the next tick) and by the
            # HTTP worker for off-schedule requests (each adds one compression to that scrape)
            "gzip_compressions": gz_where or None,
            "renders_skipped_fraction": (round(expo_events.get("render_skipped", 0) / ticks[0], 3)
                                         if ticks and ticks[0] else None),
            # compiled exposition over the run: families laid out again, segments encoded without
            # matches while the layout settled, Huffman code builds
            "exposition_events": {lab.get("event"): int(v) for _, lab, v in
                                  promtext.samples(fams, "gpuexp_exposition_events_total")} or None,
            # the same over the timed window only (steady state: relayouts should be ~0 a tick)
            "exposition_events_timed_window": ({k: int(v - expo0[k]) for k, v in
                                                list(expo_events.items()) + [("ticks", ticks[0] if ticks else 0)]
                                                if k in expo0} if expo0 else None),
            # KFD process scans over the run: directory listings vs tracked-only reads, and how
            # many processes the node's KFD proc directory holds (other GPUs' included)
            "kfd_proc_scans": {lab.get("kind"): v for _, lab, v in promtext.samples(fams, "gpuexp_kfd_proc_scans_total")}
            or None,
            "kfd_procs_tracked": next((v for _, _, v in promtext.samples(fams, "gpuexp_kfd_procs_tracked")), None),
            "http_rx_cpu_moves": next((v for _, _, v in promtext.samples(fams, "gpuexp_http_rx_cpu_moves_total")),
                                      None),
            "http_prewake_wakeups_per_scrape": round(prewake[0] / scrapes_total[0], 2)
            if prewake and scrapes_total and scrapes_total[0] else None,
            "optional_sources": {"counters": bool(args.counters), "sentinel": bool(args.sentinel),
                                 "rccl_trace": bool(rccl_dir),
                                 "degraded_reason": degraded},
            "xgmi_patterns": None,
            # --prewake-ab: per-arm latency / hit-rate / CPU table, block-bootstrap CIs against
            # the first arm, and the default the data supports (utils/abtest.py)
            "prewake_ab": abtest.analyse(ab_blocks, baseline=ab_arms[0]) if ab_arms and ab_blocks else None,
        }
    if args.xgmi_patterns and world > 1:
        patterns = xgmi_patterns(client, [b for _, _, b in pids])
        if rank == 0:
            result["xgmi_patterns"] = patterns
    if rank == 0:
        # per-peer sanity of the exporter's xGMI attribution, reported, never failing the run
        result["xgmi_checks"] = xgmi_checks(result.get("xgmi_patterns"), result.get("xgmi_timed_window"), world)
    if rank == 0:
        stop_proc(exporter)

    if args.exporter == "both":
        # Same workload, same scrape pacing, against the reference-ARCHITECTURE exporter
        # (render-on-scrape registry + vendor-library polling; utils/refstyle.py).
        ref = rclient = None
        if rank == 0:
            rport = free_port()
            cmd = [sys.executable, "-m", "kubernetes_gpu_exporter_amd.utils.refstyle", "--port", str(rport),
                   "--interval", str(1.0 / args.sample_hz), "--devices", ",".join(str(i) for i in range(n_gpus))]
            if backend == "mock":
                cmd.append("--mock")
            ref = subprocess.Popen(cmd, env=dict(os.environ, GPUEXP_POD_MAP_FILE=pod_map), cwd=ROOT,
                                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            for _ in range(600):
                try:
                    if http_get(rport, "/metrics", 0.5)[0] == 200:
                        break
                except OSError:
                    time.sleep(0.05)
            rclient = n.ScrapeClient("127.0.0.1", rport, "/metrics", args.gzip, 5000)
        if dist is not None:
            dist.barrier()
        rlat, rcpu, _ = phase(ref, rclient)
        if rank == 0:
            stop_proc(ref)
            result["refstyle"] = {"p50_scrape_us": round(statistics.median(rlat), 2) if rlat else None,
                                  "p99_scrape_us": round(pct(rlat, 0.99), 2) if rlat else None,
                                  "exporter_cpu_percent": round(rcpu, 3), "scrape_bytes": rclient.last_bytes,
                                  "scrape_errors": rclient.errors}
            if rlat and lat:
                result["speedup_p50_vs_refstyle"] = round(statistics.median(rlat) / statistics.median(lat), 2)
    problems = run_problems(result, n_gpus, attribution_ok, bool(rccl_dir)) if rank == 0 else []
    if rank == 0 and not problems:
        print(json.dumps(result), file=result_out, flush=True)
    if rank == 0 and args.out:
        extra = {"prewake_ab_blocks": abtest.blocks_to_json(ab_blocks)} if ab_blocks else {}
        with open(args.out, "w") as fh:
            json.dump(dict(result, problems=problems, **extra), fh, indent=1)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and args.mock_xgmi_file:
        try:
            os.unlink(args.mock_xgmi_file)
        except OSError:
            pass
    if problems:
        # a degraded N-GPU run must not pass for a measurement: no result line, exit 1
        for p in problems:
            print(f"[bench] FAILED: {p}", file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
