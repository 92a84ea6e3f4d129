"""Exporter configuration: one object, precedence CLI flags > env GPUEXP_* > YAML > defaults.

The reference has no configuration at all — port `:8000` (/root/reference/main.go:71),
path `/metrics` (main.go:70), interval 30 s (main.go:156), in-cluster auth only
(main.go:57) and all namespaces (main.go:77) are hard-coded.
Defaults here keep the reference's listen address and path for compatibility.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Optional

import yaml


@dataclass
class Config:
    # exposition
    listen: str = ":8000"                  # main.go:71
    path: str = "/metrics"                 # main.go:70
    http_threads: int = 1
    gzip: bool = True
    http_prewake: str = "slices"           # off | slices | spin (true = slices): have the HTTP worker awake
                                           # when a steady scraper's next request lands (HttpConfig, http.h);
                                           # default chosen by bench.py --prewake-ab (profiles/r06/prewake_ab.md)
    runtime_file: str = ""                 # YAML/JSON of run-time overrides, re-read on SIGUSR1 (http_prewake)
    stale_after: float = -1.0              # /readyz 503 when the newest sample is older (s); -1 = auto
                                           # (max(5 s, 10 intervals)), 0 = never
    # sampling
    interval: float = 1.0                  # seconds; reference: 30 s (main.go:156)
    backend: str = "auto"                  # auto | amdsmi | sysfs | mock
    device_threads: int = 0                # per-GPU read fan-out (0 = auto = serial, N > 1 = pool)
    metrics_coalesce: bool = True          # skip gpu_metrics SMU fetches until the PMFW refreshes
    metrics_min_interval: str = "auto"     # at most one gpu_metrics SMU fetch per GPU per this many s
                                           # (0 = every PMFW refresh; auto = as often as metrics_cpu_budget
                                           # allows at the measured fetch cost): bounds sampler CPU at 8 GPUs
    metrics_cpu_budget: float = 0.75       # auto: % of one core all GPUs' SMU fetches may use together
                                           # (8 loaded GPUs at 10 Hz: a fetch every 5th tick; 1 GPU: every tick)
    mock_devices: int = 1
    mock_xgmi_file: str = ""               # mock backend: per-peer traffic matrix of a CPU rehearsal (bench.py)
    host_root: str = ""                    # prefix for /sys and /proc (DaemonSet: /host)
    devices: list = field(default_factory=list)  # GPU indices and/or PCI BDFs to export (empty = all)
    series_profile: str = "full"           # full | standard (64/GPU BASELINE load) | compact | legacy
    ras_interval: float = 10.0             # seconds between RAS/AER sysfs re-reads (full profile)
    legacy_families: bool = True           # pod_gpu_memory_usage / docker_gpu_memory_perc_usage
    process_source: str = "auto"           # auto | kfd | amdsmi | none
    kfd_cu_occupancy: bool = True
    kfd_sdma_activity: bool = False        # KFD sdma_<id> per process: not SDMA time on MI355X (profiles/r04)
    kfd_detail_interval: float = 1.0       # seconds between cu_occupancy / sdma re-reads (0 = every tick)
    kfd_rescan_interval: float = 0.5       # KFD proc directory listed at least this often (also on change)
    process_min_interval: float = 0.05     # per-process reads (KFD VRAM / amdsmi list) at most this often (s;
                                           # 0 = every tick): a 100 Hz tick re-exports the last lists in between
    gc_after: int = 1
    render_when_due: bool = True           # publish a snapshot only when a steady scraper's request is due
                                           # (and >= 1/s): 15 s scrapes of a 10 Hz sampler render ~1.1/s
    exposition: str = "compiled"           # compiled (fixed-layout body, values patched in place, gzip from
                                           # pre-encoded static bits) | classic (re-render + compress)
    # optional sources
    enable_sentinel: bool = False
    sentinel_spin: int = 500
    sentinel_interval: float = 0.5         # the sentinel kernel runs at most this often (s; manual ticks: every tick)
    sentinel_impl: str = "auto"            # auto (on the PMC counters' queue when they run, else HIP) | hip | queue
    enable_counters: bool = False
    counters_plugin: str = "aqlpmc"        # aqlpmc | rocprof | /path/to/plugin.so
    counters_mode: str = "continuous"      # continuous (never paused, read every tick; aqlpmc) | duty
    counters_window_ms: int = 20           # duty: counting window ...
    counters_interval_ms: int = 1000       # ... per interval (the rocprof plugin's spin is duty-cycled)
    counters_kick: str = "auto"            # continuous: a tick's PMC read goes out at its start | after_devices |
                                           # end of the previous tick | auto (end below 50 ms ticks, else start)
    counters_min_interval: float = 0.05    # continuous counters: a PMC read round at most this often (s)
    counters_cpu_budget: float = 0.75      # continuous counters: % of one core the read rounds may use (0 = no cap)
    counters_inline: bool = True           # continuous: the sampler posts/collects each tick's PMC read itself
    http_follow_rx_cpu: bool = False       # pin the HTTP worker to the CPU a steady scraper's requests arrive on
    queue_devices: list = field(default_factory=list)  # GPUs (indices / BDFs) that get the exporter's
                                           # own GPU queue (sentinel + PMC counters); empty = all.
                                           # Each queue pins ~346 MiB of host memory on MI355X.
    enable_kfd_events: bool = True         # full profile: KFD SMI events (VM faults, resets, evictions)
    firmware_info: bool = True             # full profile: amd_gpu_firmware_info per loaded firmware
    state_file: str = ""                   # checkpoint of per-pod energy / KFD event totals ("" = off)
    state_interval: float = 10.0           # seconds between checkpoint writes (and one at shutdown)
    pod_totals_ttl: float = 3600.0         # per-pod totals of a pod absent from every (partial) pod list
                                           # this long are dropped (complete lists drop them at once)
    kfd_path: str = "/dev/kfd"             # the device node (mounted directly, not under host_root)
    enable_rccl: bool = False
    rccl_dir: str = "/var/run/gpuexp/rccl"
    rccl_verify: bool = True               # a tracer file counts only for a live process that maps it
    # attribution / kubernetes control plane
    pod_attribution: bool = True
    infer_device_owner: bool = True
    node_name: str = ""                    # downward API NODE_NAME
    kubelet_socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"
    podresources: bool = True
    # device-plugin resources that are GPUs: whole GPUs, and the partition-mode resources
    # of the AMD device plugin's "mixed" strategy (amd.com/cpx_nps4, amd.com/dpx_nps2, ...)
    gpu_resource_names: list = field(default_factory=lambda: ["amd.com/gpu", "amd.com/*px_nps*"])
    apiserver: str = ""                    # "" = in-cluster (KUBERNETES_SERVICE_HOST) if present
    apiserver_token_file: str = "/var/run/secrets/kubernetes.io/serviceaccount/token"
    apiserver_ca_file: str = "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt"
    pod_logdir: str = "/var/log/pods"      # zero-RBAC fallback: <ns>_<pod>_<uid> directories
    control_interval: float = 5.0          # seconds between control-plane refreshes
    control_timeout: float = 3.0           # per-call timeout for gRPC / apiserver
    # diagnostics
    log_level: str = "warn"
    log_format: str = "logfmt"             # logfmt | json (both the C++ core and the control plane)
    trace: str = ""                        # Chrome trace JSON of sampler stages

    def listen_host_port(self) -> tuple[str, int]:
        """(host, port).  An empty host (":8000", the reference's `ListenAndServe(":8000")`,
        main.go:71) means every interface, IPv6 and IPv4 (dual-stack, as Go binds it);
        "[::1]:8000" / "127.0.0.1:8000" bind one address."""
        host, _, port = self.listen.rpartition(":")
        if host.startswith("[") and host.endswith("]"):
            host = host[1:-1]
        if host and ":" not in host and not host.replace(".", "").isdigit():
            import socket
            try:  # a host name: the engine binds IP literals
                fam, _, _, _, addr = socket.getaddrinfo(host, None, proto=socket.IPPROTO_TCP)[0]
                host = addr[0]
            except OSError:
                pass  # left as is; validate() reports it
        return host, int(port)

    def metrics_min_interval_s(self) -> float:
        """Seconds, or -1 for auto (the engine's budget-driven cap)."""
        v = str(self.metrics_min_interval).strip().lower()
        return -1.0 if v == "auto" else float(v)

    def resolved_backend(self) -> str:
        if self.backend != "auto":
            return self.backend
        root = self.host_root or "/"
        kfd = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
        if os.path.isdir(kfd) and (os.path.exists("/dev/kfd") or self.host_root):
            return "amdsmi" if not self.host_root else "sysfs"
        return "mock"

    def to_engine_config(self, native) -> Any:
        ec = native.EngineConfig()
        ec.backend = self.resolved_backend()
        ec.mock_devices = int(self.mock_devices)
        ec.mock_xgmi_file = str(self.mock_xgmi_file)
        ec.device_threads = int(self.device_threads)
        ec.metrics_coalesce = bool(self.metrics_coalesce)
        ec.metrics_min_interval_s = self.metrics_min_interval_s()
        ec.metrics_cpu_budget = float(self.metrics_cpu_budget) / 100.0
        ec.host_root = self.host_root
        ec.interval_s = float(self.interval)
        host, port = self.listen_host_port()
        hc = native.HttpConfig()
        hc.host = host
        hc.port = port
        hc.metrics_path = self.path
        hc.threads = int(self.http_threads)
        hc.enable_gzip = bool(self.gzip)
        hc.prewake_mode = self.prewake_mode()
        hc.follow_rx_cpu = bool(self.http_follow_rx_cpu)
        stale = float(self.stale_after)
        if stale < 0:
            stale = max(5.0, 10.0 * float(self.interval)) if float(self.interval) > 0 else 0.0
        hc.stale_after_ns = int(stale * 1e9)
        ec.http = hc
        ec.series_profile = self.series_profile
        ec.ras_interval_s = float(self.ras_interval)
        ec.legacy_families = bool(self.legacy_families)
        ec.pod_attribution = bool(self.pod_attribution)
        ec.infer_device_owner = bool(self.infer_device_owner)
        ec.process_source = self.process_source
        ec.kfd_cu_occupancy = bool(self.kfd_cu_occupancy)
        ec.kfd_sdma = bool(self.kfd_sdma_activity)
        ec.kfd_detail_interval_s = float(self.kfd_detail_interval)
        ec.kfd_rescan_interval_s = float(self.kfd_rescan_interval)
        ec.process_min_interval_s = float(self.process_min_interval)
        ec.enable_sentinel = bool(self.enable_sentinel)
        ec.sentinel_spin = int(self.sentinel_spin)
        ec.sentinel_impl = str(self.sentinel_impl)
        ec.sentinel_min_interval_s = float(self.sentinel_interval)
        ec.enable_counters = bool(self.enable_counters)
        if self.counters_plugin in ("", "aqlpmc", "rocprof"):
            from ._native import rocprof_plugin_path
            ec.counters_plugin = rocprof_plugin_path(self.counters_plugin or "aqlpmc")
        else:
            ec.counters_plugin = self.counters_plugin
        ec.counters_mode = str(self.counters_mode)
        ec.counters_window_ms = int(self.counters_window_ms)
        ec.counters_interval_ms = int(self.counters_interval_ms)
        ec.counters_kick = str(self.counters_kick)
        ec.counters_inline = bool(self.counters_inline)
        ec.counters_min_interval_s = float(self.counters_min_interval)
        ec.counters_cpu_budget = float(self.counters_cpu_budget) / 100.0
        ec.enable_rccl = bool(self.enable_rccl)
        ec.rccl_dir = self.rccl_dir
        ec.rccl_verify = bool(self.rccl_verify)
        ec.enable_kfd_events = bool(self.enable_kfd_events)
        ec.firmware_info = bool(self.firmware_info)
        ec.state_file = self.state_file
        ec.state_interval_s = float(self.state_interval)
        ec.pod_totals_ttl_s = float(self.pod_totals_ttl)
        ec.kfd_path = self.kfd_path
        ec.gc_after = int(self.gc_after)
        ec.render_when_due = bool(self.render_when_due)
        ec.exposition = str(self.exposition)
        ec.device_filter = [int(d) for d in self.devices if ":" not in str(d)]
        ec.device_filter_bdf = [str(d) for d in self.devices if ":" in str(d)]
        ec.queue_devices = [int(d) for d in self.queue_devices if ":" not in str(d)]
        ec.queue_devices_bdf = [str(d) for d in self.queue_devices if ":" in str(d)]
        ec.trace_path = self.trace
        from . import __version__
        ec.version = __version__
        return ec


    def prewake_mode(self) -> str:
        return normalize_prewake(self.http_prewake)


def normalize_prewake(v: Any) -> str:
    """off | slices | spin; booleans keep their round-5 meaning (true = the timer slices)."""
    s = str(v).strip().lower()
    if s in ("", "off", "false", "0", "no"):
        return "off"
    if s in ("slices", "true", "on", "1", "yes"):
        return "slices"
    if s == "spin":
        return "spin"
    raise ValueError(f"http_prewake must be off|slices|spin, got {v!r}")


_BOOL_TRUE = {"1", "true", "yes", "on"}
_BOOL_FALSE = {"0", "false", "no", "off"}


def _coerce(f: dataclasses.Field, raw: Any) -> Any:
    default = f.default if f.default is not dataclasses.MISSING else f.default_factory()  # type: ignore
    if isinstance(default, bool):
        if isinstance(raw, bool):
            return raw
        s = str(raw).strip().lower()
        if s in _BOOL_TRUE:
            return True
        if s in _BOOL_FALSE:
            return False
        raise ValueError(f"{f.name}: not a boolean: {raw!r}")
    if isinstance(default, int):
        return int(raw)
    if isinstance(default, float):
        return float(raw)
    if isinstance(default, list):
        if isinstance(raw, (list, tuple)):
            return list(raw)
        return [x for x in str(raw).split(",") if x != ""]
    return str(raw)


# options that also work as a bare flag (`--http-prewake` = the round-5 "on")
_FLAG_CONST = {"http_prewake": "slices"}


def from_yaml(path: str) -> dict:
    with open(path) as fh:
        data = yaml.safe_load(fh) or {}
    if not isinstance(data, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    return data


def from_env(env: Optional[dict] = None) -> dict:
    env = os.environ if env is None else env
    out = {}
    for f in fields(Config):
        key = "GPUEXP_" + f.name.upper()
        if key in env:
            out[f.name] = env[key]
    if "node_name" not in out and env.get("NODE_NAME"):
        out["node_name"] = env["NODE_NAME"]
    return out


def build_arg_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="gpuexp", description="MI355X per-pod GPU Prometheus exporter")
    ap.add_argument("--config", help="YAML config file")
    for f in fields(Config):
        flag = "--" + f.name.replace("_", "-")
        default = f.default if f.default is not dataclasses.MISSING else None
        if isinstance(default, bool) or f.name in _FLAG_CONST:
            ap.add_argument(flag, dest=f.name, default=None, nargs="?", const=_FLAG_CONST.get(f.name, "true"),
                            help=f"bool (default {default})" if isinstance(default, bool) else f"(default {default!r})")
        else:
            ap.add_argument(flag, dest=f.name, default=None, help=f"(default {default!r})")
    return ap


def load_config(argv: Optional[list] = None, env: Optional[dict] = None) -> Config:
    """Merges defaults < YAML < env < CLI into one validated Config."""
    ap = build_arg_parser()
    ns = ap.parse_args(argv)
    merged: dict = {}
    if ns.config:
        merged.update(from_yaml(ns.config))
    merged.update(from_env(env))
    for f in fields(Config):
        v = getattr(ns, f.name, None)
        if v is not None:
            merged[f.name] = v
    return make_config(merged)


def make_config(values: dict) -> Config:
    known = {f.name: f for f in fields(Config)}
    kwargs = {}
    for k, v in values.items():
        k = k.replace("-", "_")
        if k not in known:
            raise ValueError(f"unknown config key: {k}")
        kwargs[k] = _coerce(known[k], v)
    cfg = Config(**kwargs)
    validate(cfg)
    return cfg


def validate(cfg: Config) -> None:
    if cfg.backend not in ("auto", "amdsmi", "sysfs", "mock"):
        raise ValueError(f"backend must be auto|amdsmi|sysfs|mock, got {cfg.backend}")
    if cfg.series_profile not in ("full", "standard", "compact", "legacy"):
        raise ValueError(f"series_profile must be full|standard|compact|legacy, got {cfg.series_profile}")
    try:
        if cfg.metrics_min_interval_s() < 0 and str(cfg.metrics_min_interval).strip().lower() != "auto":
            raise ValueError
    except ValueError:
        raise ValueError(f"metrics_min_interval must be 'auto' or seconds >= 0, got {cfg.metrics_min_interval!r}")
    if not (0 <= cfg.metrics_cpu_budget <= 100):
        raise ValueError("metrics_cpu_budget must be a percentage of one core, 0-100 (0 = no cap under auto)")
    if not (0 <= cfg.counters_cpu_budget <= 100):
        raise ValueError("counters_cpu_budget must be a percentage of one core, 0-100 (0 = no cap)")
    normalize_prewake(cfg.http_prewake)
    if cfg.exposition not in ("compiled", "classic"):
        raise ValueError(f"exposition must be compiled|classic, got {cfg.exposition}")
    if cfg.counters_kick not in ("auto", "start", "after_devices", "end"):
        raise ValueError(f"counters_kick must be auto|start|after_devices|end, got {cfg.counters_kick}")
    if cfg.state_interval <= 0:
        raise ValueError("state_interval must be > 0")
    if cfg.pod_totals_ttl <= 0:
        raise ValueError("pod_totals_ttl must be > 0")
    if cfg.process_min_interval < 0:
        raise ValueError("process_min_interval must be >= 0 seconds")
    if cfg.ras_interval <= 0:
        raise ValueError("ras_interval must be > 0")
    if cfg.process_source not in ("auto", "kfd", "amdsmi", "none"):
        raise ValueError(f"process_source must be auto|kfd|amdsmi|none, got {cfg.process_source}")
    if cfg.interval < 0 or (0 < cfg.interval < 0.001):
        raise ValueError("interval must be 0 (manual) or >= 1 ms")
    if not cfg.path.startswith("/"):
        raise ValueError("path must start with /")
    _, port = cfg.listen_host_port()
    if not (0 <= port < 65536):
        raise ValueError("listen port out of range")
    if cfg.mock_devices < 1:
        raise ValueError("mock_devices must be >= 1")
    if cfg.log_level not in ("debug", "info", "warn", "error", "off"):
        raise ValueError("log_level must be debug|info|warn|error|off")
    if cfg.log_format not in ("logfmt", "json"):
        raise ValueError("log_format must be logfmt|json")
    if cfg.sentinel_impl not in ("auto", "hip", "queue"):
        raise ValueError(f"sentinel_impl must be auto|hip|queue, got {cfg.sentinel_impl}")
    if cfg.counters_mode not in ("continuous", "duty"):
        raise ValueError(f"counters_mode must be continuous|duty, got {cfg.counters_mode}")
    if cfg.stale_after < 0 and cfg.stale_after != -1:
        raise ValueError("stale_after must be -1 (auto), 0 (never) or > 0 seconds")
    host, _ = cfg.listen_host_port()
    if host and ":" not in host:
        import ipaddress
        try:
            ipaddress.IPv4Address(host)
        except ValueError:
            try:  # a name, as Go's net.Listen accepts: resolved once, here
                import socket
                socket.getaddrinfo(host, None)
            except OSError:
                raise ValueError(f"listen host {host!r} is neither an IP address nor a resolvable name")
