"""Process entry point: wires the native engine to the Kubernetes control plane.

Reference lifecycle (/root/reference/main.go:38-158): register two GaugeVecs, nvml.Init
(fatal on error), rest.InClusterConfig (panic outside a cluster), start the HTTP
goroutine, then loop forever; `nvml.Shutdown` is deferred but never runs.
Here: the native engine owns sampling + serving; a Python control-plane thread refreshes
pod metadata at low rate; SIGTERM/SIGINT stop both and shut amdsmi/HIP down cleanly.
"""
from __future__ import annotations

import logging
import os
import signal
import threading
from typing import Optional

from ._native import load
from .config import Config

log = logging.getLogger("gpuexp")

_LEVELS = {"debug": 0, "info": 1, "warn": 2, "error": 3, "off": 4}


class Exporter:
    def __init__(self, cfg: Config, control_plane: Optional[object] = None):
        self.cfg = cfg
        self.native = load()
        self.native.set_log_level(_LEVELS[cfg.log_level])
        self.native.set_log_json(cfg.log_format == "json")
        self.engine = self.native.Engine(cfg.to_engine_config(self.native))
        self._control = control_plane
        self._stop = threading.Event()
        self._started = False

    # ---- lifecycle ----
    def start(self) -> "Exporter":
        self.engine.start()
        self._started = True
        # The mock backend gets a control plane only from an explicit pod map (bench, tests):
        # it must never pick up a real node's kubelet or apiserver.
        if self._control is None and self.cfg.pod_attribution and (
                self.cfg.resolved_backend() != "mock" or os.environ.get("GPUEXP_POD_MAP_FILE")):
            from .k8s.controlplane import ControlPlane
            self._control = ControlPlane.from_config(self.cfg)
        if self._control is not None:
            self._control.attach(self.engine)
            self._control.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._control is not None:
            self._control.stop()
        if self._started:
            self.engine.stop()
            self._started = False

    def __enter__(self) -> "Exporter":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    # ---- accessors ----
    @property
    def port(self) -> int:
        return self.engine.http_port

    def text(self) -> str:
        return self.engine.snapshot_text()

    def tick(self, now_ns: Optional[int] = None) -> None:
        self.engine.tick(now_ns)

    def stats(self) -> dict:
        return self.engine.stats()

    def apply_runtime(self, path: Optional[str] = None) -> dict:
        """Applies the run-time overrides file (config `runtime_file`, re-read on SIGUSR1):
        a YAML/JSON mapping; supported key: `http_prewake` (off|slices|spin).  Returns what
        was applied; a bad file is logged and changes nothing."""
        path = path or self.cfg.runtime_file
        if not path:
            return {}
        from .config import from_yaml, normalize_prewake
        try:
            data = from_yaml(path)
            applied = {}
            if "http_prewake" in data:
                mode = normalize_prewake(data["http_prewake"])
                if self.engine.set_prewake_mode(mode):
                    applied["http_prewake"] = mode
            unknown = sorted(set(data) - {"http_prewake"})
            if unknown:
                log.warning("runtime file %s: ignored keys %s", path, unknown)
            return applied
        except (OSError, ValueError) as ex:
            log.warning("runtime file %s not applied: %s", path, ex)
            return {}

    def run_forever(self) -> int:
        def _handler(signum, frame):
            log.info("signal %s: shutting down", signum)
            self._stop.set()

        def _refresh(signum, frame):
            if self._control is not None and hasattr(self._control, "refresh_soon"):
                self._control.refresh_soon()

        signal.signal(signal.SIGTERM, _handler)
        signal.signal(signal.SIGINT, _handler)
        signal.signal(signal.SIGHUP, _refresh)  # re-read pod metadata now
        signal.signal(signal.SIGUSR1, lambda signum, frame: self.apply_runtime())  # run-time overrides
        self.start()
        log.info("serving %s on %s (%s)", self.cfg.path, self.cfg.listen, self.engine.source_status())
        # no timeout: lock waits are interrupted by signals, the handler sets the event, and
        # the main thread wakes only then (a 1 s poll cost a wake-up per second for nothing)
        self._stop.wait()
        self.stop()
        return 0
