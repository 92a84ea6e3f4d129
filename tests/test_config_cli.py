"""Config precedence (CLI > env > YAML > defaults), validation, and the CLI daemon end to
end: start, serve, SIGTERM -> clean exit (the reference's deferred nvml.Shutdown never ran,
/root/reference/main.go:49-54)."""
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

from kubernetes_gpu_exporter_amd.config import Config, load_config, make_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defaults_match_reference_endpoint():
    c = Config()
    assert c.listen == ":8000" and c.path == "/metrics"  # main.go:70-71
    assert c.listen_host_port() == ("", 8000)  # all interfaces, dual-stack like Go's ":8000"


def test_precedence(tmp_path):
    y = tmp_path / "c.yaml"
    y.write_text("interval: 5\nlisten: ':9000'\nenable_sentinel: true\nmock_devices: 3\n")
    env = {"GPUEXP_INTERVAL": "2", "GPUEXP_MOCK_DEVICES": "4", "NODE_NAME": "node-7"}
    c = load_config(["--config", str(y), "--interval", "0.5"], env=env)
    assert c.interval == 0.5            # CLI
    assert c.mock_devices == 4          # env over YAML
    assert c.listen == ":9000"          # YAML
    assert c.enable_sentinel is True
    assert c.node_name == "node-7"      # downward API
    c = load_config(["--gzip", "false", "--devices", "0,2"], env={})
    assert c.gzip is False and c.devices == ["0", "2"]
    c = load_config(["--enable-counters"], env={})  # bare flag = true
    assert c.enable_counters is True


@pytest.mark.parametrize("bad", [
    {"backend": "nvml"}, {"series_profile": "huge"}, {"interval": -1}, {"path": "metrics"},
    {"listen": ":99999"}, {"mock_devices": 0}, {"log_level": "loud"}, {"nonsense": 1}, {"gzip": "maybe"},
    {"exposition": "fast"},
])
def test_validation(bad):
    with pytest.raises(ValueError):
        make_config(bad)


def test_engine_config_translation(native):
    c = make_config({"listen": "127.0.0.1:9123", "path": "/m", "backend": "mock", "interval": 0.1,
                     "devices": "1,3", "series_profile": "compact"})
    ec = c.to_engine_config(native)
    assert (ec.http.host, ec.http.port, ec.http.metrics_path) == ("127.0.0.1", 9123, "/m")
    assert ec.backend == "mock" and ec.interval_s == 0.1 and ec.device_filter == [1, 3]
    assert ec.series_profile == "compact"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cli_daemon_lifecycle(tmp_path):
    port = _free_port()
    trace = tmp_path / "trace.json"
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--backend", "mock",
                          "--mock-devices", "2", "--listen", f"127.0.0.1:{port}", "--path", "/custom",
                          "--interval", "0.02", "--trace", str(trace)],
                         cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        body = None
        for _ in range(200):
            try:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/custom", timeout=1).read().decode()
                break
            except Exception:
                time.sleep(0.05)
        assert body and 'amd_gpu_up{gpu="1"' in body
        time.sleep(0.2)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=15) == 0
    finally:
        if p.poll() is None:
            p.kill()
    import json
    events = [e for e in json.loads(trace.read_text()) if e]
    assert {e["name"] for e in events} >= {"devices", "processes", "render"}


def test_cli_sighup_refreshes_instead_of_exiting(tmp_path):
    """SIGHUP asks the control plane to re-read pod metadata now (the bench sends it after
    writing its pod map); the daemon keeps serving and still exits cleanly on SIGTERM."""
    port = _free_port()
    pod_map = tmp_path / "pods.json"
    pod_map.write_text('{"pods": [], "pid_cgroups": {}, "device_owners": {}}')
    env = dict(os.environ, GPUEXP_POD_MAP_FILE=str(pod_map))
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_gpu_exporter_amd", "--backend", "mock",
                          "--listen", f"127.0.0.1:{port}", "--interval", "0.05", "--control-interval", "60"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        for _ in range(200):
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=1).read()
                break
            except Exception:
                time.sleep(0.05)
        p.send_signal(signal.SIGHUP)
        time.sleep(0.3)
        assert p.poll() is None
        assert urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=1).status == 200
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=15) == 0
    finally:
        if p.poll() is None:
            p.kill()


def test_control_plane_refresh_soon():
    from kubernetes_gpu_exporter_amd.k8s.controlplane import ControlPlane, Metadata

    class _Src:
        name = "src"

        def fetch(self):
            return Metadata()

    cp = ControlPlane([_Src()], interval=60.0)
    cp.start()
    try:
        n0 = cp.refreshes
        time.sleep(0.1)
        assert cp.refreshes == n0  # the interval has not passed
        cp.refresh_soon()
        for _ in range(100):
            if cp.refreshes > n0:
                break
            time.sleep(0.01)
        assert cp.refreshes == n0 + 1
    finally:
        cp.stop()


def test_round4_keys_reach_the_engine(native):
    from kubernetes_gpu_exporter_amd.config import make_config
    ec = make_config({}).to_engine_config(native)
    assert ec.counters_inline is True and ec.http.follow_rx_cpu is False and ec.kfd_sdma is False
    ec = make_config({"counters_inline": False, "http_follow_rx_cpu": True,
                      "kfd_sdma_activity": True}).to_engine_config(native)
    assert ec.counters_inline is False and ec.http.follow_rx_cpu is True and ec.kfd_sdma is True


def test_round5_keys_reach_the_engine(native):
    ec = make_config({}).to_engine_config(native)
    # pre-wake on (slices) since round 6's in-process A/B (profiles/r06/prewake_ab.md)
    assert ec.exposition == "compiled" and ec.http.prewake is True and ec.http.prewake_mode == "slices"
    c = load_config(["--http-prewake", "false"], env={"GPUEXP_EXPOSITION": "classic"})
    assert c.to_engine_config(native).http.prewake is False
    c = load_config(["--http-prewake"], env={"GPUEXP_EXPOSITION": "classic"})
    ec = c.to_engine_config(native)
    assert ec.exposition == "classic" and ec.http.prewake is True


def test_stale_after_defaults_follow_the_interval(native):
    from kubernetes_gpu_exporter_amd.config import make_config
    def ns(**kw):
        return make_config(kw).to_engine_config(native).http.stale_after_ns
    assert ns(interval=0.1) == 5_000_000_000      # at least 5 s
    assert ns(interval=1.0) == 10_000_000_000     # 10 intervals
    assert ns(interval=0) == 0                    # manual ticks: never stale
    assert ns(interval=1.0, stale_after=2) == 2_000_000_000
    assert ns(interval=1.0, stale_after=0) == 0


def test_listen_and_stale_after_validation():
    from kubernetes_gpu_exporter_amd.config import make_config
    assert make_config({"listen": "[::1]:9000"}).listen_host_port() == ("::1", 9000)
    assert make_config({"listen": "127.0.0.1:9000"}).listen_host_port() == ("127.0.0.1", 9000)
    assert make_config({"listen": "localhost:9000"}).listen_host_port()[0] in ("127.0.0.1", "::1")
    for bad in ({"listen": "no-such-host.invalid:9000"}, {"stale_after": -5}):
        with pytest.raises(ValueError):
            make_config(bad)


def test_python_logs_are_logfmt_like_the_core(capsys):
    """Control-plane log lines use the C++ core's logfmt (csrc/gpuexp/common.cc)."""
    import logging
    import re

    from kubernetes_gpu_exporter_amd.utils import logfmt
    logfmt.setup("info")
    try:
        logging.getLogger("gpuexp.control").warning('source "x" failed:\nboom \\ done')
        logging.getLogger("gpuexp").debug("hidden at info")
    finally:
        logfmt.setup("warn")
    err = capsys.readouterr().err.strip().splitlines()
    assert len(err) == 1, err
    assert re.fullmatch(r'ts=\d+\.\d{3} level=warn component=control msg="source \\"x\\" failed: boom \\\\ done"',
                        err[0]), err[0]


def test_json_log_format_from_both_halves(capfd, native):
    """log_format=json: the C++ core and the Python control plane both write one JSON object
    per line with the same keys (escaped quotes, backslashes and control characters)."""
    import json
    import logging

    from kubernetes_gpu_exporter_amd.utils import logfmt
    assert make_config({"log_format": "json"}).log_format == "json"
    with pytest.raises(ValueError):
        make_config({"log_format": "xml"})
    logfmt.setup("info", "json")
    native.set_log_json(True)
    try:
        native.log(2, "sampler", 'gpu "0" \\ read\x01failed\nretrying')
        logging.getLogger("gpuexp.control").warning('source "x"\nfailed')
    finally:
        native.set_log_json(False)
        logfmt.setup("warn")
    lines = [l for l in capfd.readouterr().err.splitlines() if l.strip()]
    recs = [json.loads(l) for l in lines]
    assert [sorted(r) for r in recs] == [["component", "level", "msg", "ts"]] * 2, lines
    core, py = recs
    assert core["component"] == "sampler" and core["level"] == "warn"
    assert core["msg"] == 'gpu "0" \\ read\x01failed retrying'
    assert py["component"] == "control" and py["msg"] == 'source "x" failed'
    assert abs(core["ts"] - py["ts"]) < 60


def test_round6_prewake_modes(native):
    """http_prewake is a mode (off|slices|spin); booleans keep their round-5 meaning and the
    bare flag is the timer-slice mode.  The engine's HttpConfig carries it as prewake_mode."""
    from kubernetes_gpu_exporter_amd.config import normalize_prewake
    assert normalize_prewake(True) == "slices" and normalize_prewake(False) == "off"
    assert normalize_prewake("SPIN") == "spin"
    with pytest.raises(ValueError):
        make_config({"http_prewake": "busy"})
    for argv, want in ((["--http-prewake"], "slices"), (["--http-prewake", "spin"], "spin"),
                       (["--http-prewake", "false"], "off")):
        ec = load_config(argv, env={}).to_engine_config(native)
        assert ec.http.prewake_mode == want, argv
    ec = make_config({"http_prewake": "spin"}).to_engine_config(native)
    assert ec.http.prewake is True  # the legacy boolean view: any mode but off
    c = native.HttpConfig()
    c.prewake = True
    assert c.prewake_mode == "slices"
    with pytest.raises(ValueError):
        c.prewake_mode = "nope"
