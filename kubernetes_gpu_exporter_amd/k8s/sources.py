"""Pod-metadata sources for the control plane.

ApiserverSource replaces the reference's cluster-wide `Pods("").List` every cycle
(/root/reference/main.go:77, all namespaces, all nodes, panic on error) with a
NODE-SCOPED list (fieldSelector=spec.nodeName=$NODE_NAME, served from the watch cache via
resourceVersion=0) over plain HTTPS with the ServiceAccount token — no client library,
per-call timeout, errors isolated.  Container IDs have their `<runtime>://` scheme removed
correctly (the reference's Index("://")+3 sliced from offset 2 when absent, main.go:97).

LogdirSource needs no RBAC at all: kubelet names pod log directories
/var/log/pods/<namespace>_<pod>_<uid>/<container>/.
"""
from __future__ import annotations

import json
import os
import ssl
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


def pods_from_list(obj: dict) -> Metadata:
    md = Metadata()
    for item in obj.get("items", []):
        meta = item.get("metadata", {})
        uid = meta.get("uid", "")
        if not uid:
            continue
        containers = {}
        st = item.get("status", {})
        for key in ("containerStatuses", "initContainerStatuses", "ephemeralContainerStatuses"):
            for cs in st.get(key, []) or []:
                cid = strip_container_id(cs.get("containerID", ""))
                if cid:
                    containers[cid.lower()] = cs.get("name", "")
        md.pods[uid] = {"uid": uid, "namespace": meta.get("namespace", ""), "name": meta.get("name", ""),
                        "containers": containers}
    return md


class ApiserverSource(Source):
    name = "apiserver"

    def __init__(self, base_url: str, node_name: str, token_file: str = "", ca_file: str = "",
                 timeout: float = 3.0, insecure: bool = False):
        self.base_url = base_url.rstrip("/")
        self.node_name = node_name
        self.token_file = token_file
        self.ca_file = ca_file
        self.timeout = timeout
        self.insecure = insecure
        self.requests = 0

    @classmethod
    def from_config(cls, cfg):
        base = cfg.apiserver
        if not base:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
            if not host:
                return None
            base = f"https://{host}:{port or 443}"
        return cls(base, cfg.node_name, cfg.apiserver_token_file, cfg.apiserver_ca_file, cfg.control_timeout)

    def _url(self) -> str:
        q = {"resourceVersion": "0"}
        if self.node_name:
            q["fieldSelector"] = f"spec.nodeName={self.node_name}"
        return f"{self.base_url}/api/v1/pods?{urllib.parse.urlencode(q)}"

    def fetch(self) -> Metadata:
        req = urllib.request.Request(self._url(), headers={"Accept": "application/json"})
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
        with urllib.request.urlopen(req, timeout=self.timeout, context=ctx) as r:
            obj = json.loads(r.read())
        return pods_from_list(obj)


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
