"""Control plane: merges pod-metadata sources and pushes them into the native engine.

Reference: every 30 s it listed ALL pods cluster-wide (/root/reference/main.go:77) and ran
`kubectl exec <pod> -- ps` per container status (main.go:92-110), serially, with no
timeout, on the collection path.  Here metadata is refreshed off the sampling path, at
low rate, only pushed when it changed, with per-source timeouts and error isolation:

  PodResourcesSource  kubelet gRPC  -> device (BDF/UUID) -> owning pod/container
  ApiserverSource     node-scoped list + watch -> pod UID -> namespace/name, container IDs
  LogdirSource        /var/log/pods/<ns>_<pod>_<uid>  (zero-RBAC fallback)
  FileSource          JSON map (tests, bench, non-Kubernetes schedulers)
"""
from __future__ import annotations

import json
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

log = logging.getLogger("gpuexp.control")


@dataclass
class Metadata:
    pods: dict = field(default_factory=dict)         # uid -> {uid, namespace, name, containers{cid: name}}
    owners: dict = field(default_factory=dict)       # bdf|uuid -> {namespace, pod, container}
    pid_cgroups: dict = field(default_factory=dict)  # pid -> cgroup path (tests / non-hostPID setups)

    def merge(self, other: "Metadata") -> None:
        for uid, p in other.pods.items():
            cur = self.pods.get(uid)
            if cur is None:
                self.pods[uid] = dict(p, containers=dict(p.get("containers", {})))
            else:
                cur.update({k: v for k, v in p.items() if k != "containers" and v})
                cur.setdefault("containers", {}).update(p.get("containers", {}))
        self.owners.update(other.owners)
        self.pid_cgroups.update(other.pid_cgroups)

    def fingerprint(self) -> str:
        return json.dumps([self.pods, self.owners, {str(k): v for k, v in self.pid_cgroups.items()}],
                          sort_keys=True)


class Source:
    name = "source"

    def fetch(self) -> Metadata:  # pragma: no cover - interface
        """The source's current metadata.  A source may return the same object as last time
        only if nothing changed (the control plane then skips the refresh); a change must come
        as a new object, never by mutating the one handed out before."""
        raise NotImplementedError

    @property
    def has_synced(self) -> bool:
        """False while the source has never produced a complete answer (e.g. the apiserver
        list has not succeeded yet): its (empty) pods are then not a statement that pods
        are gone."""
        return True

    def close(self) -> None:
        """Releases background resources (watch threads, channels)."""


class ControlPlane:
    def __init__(self, sources: list, interval: float = 5.0):
        # Lowest priority first; later sources override earlier ones on conflicts.
        self.sources = list(sources)
        self.interval = interval
        self.engine = None
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._kick = threading.Event()  # refresh_soon(): refresh now instead of at the interval
        self._last_fp = None
        self._pushed_pids: set = set()
        self.errors: dict = {}
        self.refreshes = 0
        self.last_complete = False
        self._last_fetched: Optional[list] = None
        self._last_md: Optional[Metadata] = None

    @classmethod
    def from_config(cls, cfg) -> "ControlPlane":
        import os
        from .sources import ApiserverSource, LogdirSource, PodResourcesSource
        from .filesource import FileSource
        root = cfg.host_root.rstrip("/")
        srcs: list = []
        logdir = root + cfg.pod_logdir if root else cfg.pod_logdir
        if os.path.isdir(logdir):
            srcs.append(LogdirSource(logdir))
        api = ApiserverSource.from_config(cfg)
        if api is not None:
            srcs.append(api)
        sock = root + cfg.kubelet_socket if root else cfg.kubelet_socket
        if cfg.podresources and os.path.exists(sock):
            srcs.append(PodResourcesSource(sock, cfg.gpu_resource_names, timeout=cfg.control_timeout))
        pod_map = os.environ.get("GPUEXP_POD_MAP_FILE")
        if pod_map:
            srcs.append(FileSource(pod_map))
        return cls(srcs, cfg.control_interval)

    def attach(self, engine) -> None:
        self.engine = engine

    def refresh_once(self) -> Metadata:
        md = Metadata()
        complete = True  # every source answered: only then may the engine drop per-pod totals
        fetched: list = []
        for s in self.sources:
            try:
                got = s.fetch()
                fetched.append((got, bool(getattr(s, "has_synced", True)), getattr(s, "last_error", None)))
            except Exception as e:  # one failing source never blocks the others
                fetched.append((None, False, e))
        # Sources that cache (FileSource between file changes) hand back the very objects of
        # the last refresh: nothing can have changed, so skip the merge and the fingerprint
        # (the refresh then costs a stat per source; the bench refreshes every 0.5 s).  The
        # previous objects are held, so their ids cannot be reused by new ones.
        if self._last_fetched is not None and len(fetched) == len(self._last_fetched) and all(
                a[0] is not None and a[0] is b[0] and a[1:] == b[1:] for a, b in zip(fetched, self._last_fetched)):
            self.refreshes += 1
            return self._last_md
        for s, (got, synced, err) in zip(self.sources, fetched):
            try:
                if got is None:
                    raise err
                md.merge(got)
                complete = complete and synced
                # a source may keep serving its cache while its background loop fails
                err = getattr(s, "last_error", None)
                if err:
                    self.errors[s.name] = err
                else:
                    self.errors.pop(s.name, None)
            except Exception as e:  # one failing source never blocks the others
                complete = False
                self.errors[s.name] = repr(e)
                log.warning("source %s failed: %r", s.name, e)
        self.last_complete = complete
        fp = md.fingerprint() + ("" if complete else "#partial")
        if self.engine is not None and fp != self._last_fp:
            self.engine.set_pods(list(md.pods.values()), complete)
            self.engine.set_device_owners(md.owners)
            pids = {int(p) for p in md.pid_cgroups}
            if self._pushed_pids - pids:
                self.engine.clear_pid_cgroups()
            for pid, path in md.pid_cgroups.items():
                self.engine.set_pid_cgroup(int(pid), path)
            self._pushed_pids = pids
            self._last_fp = fp
        self._last_fetched = fetched
        self._last_md = md
        self.refreshes += 1
        return md

    def _run(self) -> None:
        while not self._stop.is_set():
            t0 = time.monotonic()
            self.refresh_once()
            self._kick.wait(max(0.05, self.interval - (time.monotonic() - t0)))
            self._kick.clear()

    def start(self) -> None:
        self.refresh_once()
        self._thread = threading.Thread(target=self._run, name="gpuexp-control", daemon=True)
        self._thread.start()

    def refresh_soon(self) -> None:
        """Refreshes at once instead of at the next interval (SIGHUP to the exporter: e.g. a
        pod map file rewritten by a scheduler, or an operator who wants new pods now)."""
        self._kick.set()

    def stop(self) -> None:
        self._stop.set()
        self._kick.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        for s in self.sources:
            try:
                s.close()
            except Exception as e:  # pragma: no cover - best effort at shutdown
                log.warning("closing source %s: %r", s.name, e)
