"""Pod-metadata sources for the control plane.

ApiserverSource replaces the reference's cluster-wide `Pods("").List` every cycle
(/root/reference/main.go:77, all namespaces, all nodes, panic on error) with an
informer-style NODE-SCOPED list + watch (fieldSelector=spec.nodeName=$NODE_NAME) over
plain HTTPS with the ServiceAccount token — no client library: one list (served from the
watch cache, resourceVersion=0), then a streaming watch that applies ADDED / MODIFIED /
DELETED events to a local cache and resumes from the last resourceVersion (BOOKMARKs keep
it fresh); 410 Gone -> relist; errors -> capped exponential backoff.  fetch() reads the
cache, so a control-plane refresh costs no apiserver request at all.  Container IDs have their `<runtime>://` scheme removed
correctly (the reference's Index("://")+3 sliced from offset 2 when absent, main.go:97).

LogdirSource needs no RBAC at all: kubelet names pod log directories
/var/log/pods/<namespace>_<pod>_<uid>/<container>/.
"""
from __future__ import annotations

import json
import logging
import os
import ssl
import threading
import time
import urllib.error
import urllib.parse
import urllib.request

from .controlplane import Metadata, Source
from .podresources import PodResourcesSource  # noqa: F401  (re-export)


def strip_container_id(cid: str) -> str:
    """'containerd://abc' -> 'abc'; 'abc' -> 'abc' (reference bug Q13 fixed)."""
    if not cid:
        return ""
    i = cid.find("://")
    return cid[i + 3:] if i >= 0 else cid


def pod_entry(item: dict) -> dict | None:
    meta = item.get("metadata", {})
    uid = meta.get("uid", "")
    if not uid:
        return None
    containers = {}
    st = item.get("status", {})
    for key in ("containerStatuses", "initContainerStatuses", "ephemeralContainerStatuses"):
        for cs in st.get(key, []) or []:
            cid = strip_container_id(cs.get("containerID", ""))
            if cid:
                containers[cid.lower()] = cs.get("name", "")
    return {"uid": uid, "namespace": meta.get("namespace", ""), "name": meta.get("name", ""),
            "containers": containers}


def pods_from_list(obj: dict) -> Metadata:
    md = Metadata()
    for item in obj.get("items", []):
        e = pod_entry(item)
        if e is not None:
            md.pods[e["uid"]] = e
    return md


log = logging.getLogger("gpuexp.apiserver")


class ApiserverSource(Source):
    name = "apiserver"

    def __init__(self, base_url: str, node_name: str, token_file: str = "", ca_file: str = "",
                 timeout: float = 3.0, insecure: bool = False, watch: bool = True, watch_timeout_s: int = 300):
        self.base_url = base_url.rstrip("/")
        self.node_name = node_name
        self.token_file = token_file
        self.ca_file = ca_file
        self.timeout = timeout
        self.insecure = insecure
        self.watch = watch
        self.watch_timeout_s = int(watch_timeout_s)
        self.requests = 0          # HTTP requests issued (lists + watches)
        self.relists = 0
        self.events = 0
        self._pods: dict = {}      # uid -> pod entry
        self._rv = ""
        self._synced = False
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._resp = None          # open watch response (closed by close())
        self.last_error = None     # set while the watch loop is failing (reported, cache kept)

    @classmethod
    def from_config(cls, cfg):
        base = cfg.apiserver
        if not base:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
            if not host:
                return None
            base = f"https://{host}:{port or 443}"
        return cls(base, cfg.node_name, cfg.apiserver_token_file, cfg.apiserver_ca_file, cfg.control_timeout)

    # --- HTTP ---
    def _url(self, **extra) -> str:
        q = {}
        if self.node_name:
            q["fieldSelector"] = f"spec.nodeName={self.node_name}"
        q.update(extra)
        return f"{self.base_url}/api/v1/pods?{urllib.parse.urlencode(q)}"

    def _open(self, url: str, timeout: float):
        req = urllib.request.Request(url, headers={"Accept": "application/json"})
        if self.token_file and os.path.exists(self.token_file):
            with open(self.token_file) as fh:
                req.add_header("Authorization", "Bearer " + fh.read().strip())
        ctx = None
        if self.base_url.startswith("https"):
            ctx = ssl.create_default_context(cafile=self.ca_file if self.ca_file and os.path.exists(self.ca_file) else None)
            if self.insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
        self.requests += 1
        return urllib.request.urlopen(req, timeout=timeout, context=ctx)

    def _list(self) -> None:
        with self._open(self._url(resourceVersion="0"), self.timeout) as r:
            obj = json.loads(r.read())
        pods = {}
        for item in obj.get("items", []):
            e = pod_entry(item)
            if e is not None:
                pods[e["uid"]] = e
        with self._lock:
            self._pods = pods
            self._rv = obj.get("metadata", {}).get("resourceVersion", "")
            self._synced = True
        self.relists += 1

    def _apply(self, ev: dict) -> bool:
        """Applies one watch event; returns False when the watch must relist (410 Gone)."""
        typ = ev.get("type", "")
        obj = ev.get("object", {}) or {}
        if typ == "ERROR":
            if obj.get("code") == 410:
                return False
            raise RuntimeError(f"watch error: {obj.get('message', obj)}")
        rv = obj.get("metadata", {}).get("resourceVersion", "")
        with self._lock:
            if typ in ("ADDED", "MODIFIED"):
                e = pod_entry(obj)
                if e is not None:
                    self._pods[e["uid"]] = e
            elif typ == "DELETED":
                self._pods.pop(obj.get("metadata", {}).get("uid", ""), None)
            if rv:
                self._rv = rv
        self.events += 1
        return True

    def _watch_once(self) -> bool:
        """One streaming watch from the current resourceVersion; returns False on 410."""
        url = self._url(watch="1", resourceVersion=self._rv, allowWatchBookmarks="true",
                        timeoutSeconds=str(self.watch_timeout_s))
        try:
            r = self._open(url, self.watch_timeout_s + self.timeout)
        except urllib.error.HTTPError as e:
            if e.code == 410:
                return False
            raise
        self._resp = r
        try:
            while not self._stop.is_set():
                line = r.readline()
                if not line:
                    return True  # server closed (timeoutSeconds): resume from rv
                line = line.strip()
                if line and not self._apply(json.loads(line)):
                    return False
        finally:
            self._resp = None
            r.close()
        return True

    def _run(self) -> None:
        backoff = 0.5
        while not self._stop.is_set():
            try:
                if not self._synced:
                    self._list()
                self.last_error = None
                if not self._watch_once():
                    self._synced = False  # 410 Gone: history compacted, relist
                backoff = 0.5
            except Exception as e:  # network, auth, decode: back off, then resume/relist
                if self._stop.is_set():
                    break
                self.last_error = repr(e)
                log.warning("apiserver watch failed: %r (retry in %.1fs)", e, backoff)
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 30.0)
                self._synced = False

    # --- Source ---
    @property
    def has_synced(self) -> bool:
        return self.relists > 0  # the node's pod list has been read in full at least once

    def fetch(self) -> Metadata:
        if not self.watch:
            self._list()
        elif self._thread is None:
            self._list()  # first call: synchronous list, so the first refresh has names
            self._thread = threading.Thread(target=self._run, name="gpuexp-apiserver-watch", daemon=True)
            self._thread.start()
        # While the watch relists (410 / reconnect) the last cache is served: stale names for
        # a moment beat pods vanishing from the exposition.
        md = Metadata()
        with self._lock:
            md.pods = {uid: dict(p, containers=dict(p["containers"])) for uid, p in self._pods.items()}
        return md

    def close(self) -> None:
        self._stop.set()
        r = self._resp
        if r is not None:
            # Unblock a readline() parked in the watch stream: shut the socket down
            # (closing the response object from another thread does not wake recv()).
            try:
                import socket as _socket
                r.fp.raw._sock.shutdown(_socket.SHUT_RDWR)
            except Exception:
                pass
        if self._thread is not None:
            self._thread.join(timeout=5)


class LogdirSource(Source):
    name = "logdir"

    def __init__(self, path: str):
        self.path = path

    def fetch(self) -> Metadata:
        md = Metadata()
        try:
            entries = os.listdir(self.path)
        except OSError:
            return md
        for e in entries:
            parts = e.split("_")
            if len(parts) < 3:
                continue
            ns, uid = parts[0], parts[-1]
            name = "_".join(parts[1:-1])
            if len(uid) != 36 or uid.count("-") != 4:
                continue
            md.pods[uid] = {"uid": uid, "namespace": ns, "name": name, "containers": {}}
        return md
