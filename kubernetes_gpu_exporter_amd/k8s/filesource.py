"""JSON pod-map source: {"pods": [{uid, namespace, name, containers{cid: name}}],
"device_owners": {bdf|uuid: {namespace, pod, container}}, "pid_cgroups": {pid: path}}.
Reloaded when the file's mtime changes.  Used by the benchmark (to attribute synthetic
workload ranks to fake pods) and for schedulers other than Kubernetes."""
from __future__ import annotations

import json
import os

from .controlplane import Metadata, Source


class FileSource(Source):
    name = "file"

    def __init__(self, path: str):
        self.path = path
        self._mtime = None
        self._md = Metadata()

    def fetch(self) -> Metadata:
        try:
            st = os.stat(self.path)
        except FileNotFoundError:
            return Metadata()
        if st.st_mtime_ns != self._mtime:
            with open(self.path) as fh:
                data = json.load(fh)
            md = Metadata()
            for p in data.get("pods", []):
                md.pods[p["uid"]] = {"uid": p["uid"], "namespace": p.get("namespace", ""),
                                     "name": p.get("name", ""), "containers": dict(p.get("containers", {}))}
            md.owners = dict(data.get("device_owners", {}))
            md.pid_cgroups = {int(k): v for k, v in data.get("pid_cgroups", {}).items()}
            self._md = md
            self._mtime = st.st_mtime_ns
        return self._md


def write_pod_map(path: str, pods: list, pid_cgroups: dict | None = None, owners: dict | None = None) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        json.dump({"pods": pods, "pid_cgroups": {str(k): v for k, v in (pid_cgroups or {}).items()},
                   "device_owners": owners or {}}, fh)
    os.replace(tmp, path)
