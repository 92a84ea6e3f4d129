"""Fakes for the Kubernetes control plane (there is no cluster in CI or on the GPU box).

FakeKubelet    — PodResources v1 gRPC server on a unix socket (same wire format as the
                 kubelet: `/v1.PodResourcesLister/List`).
FakeApiserver  — HTTP server for GET /api/v1/pods (list and ?watch=1 event stream) with
                 fieldSelector=spec.nodeName, bearer-token auth, resourceVersions,
                 bookmarks and 410-Gone injection, shaped like the real thing.
FakePod        — one pod: uid, namespace, name, node, containers {name: container_id},
                 GPUs {container_name: [device_ids]}.
"""
from __future__ import annotations

import json
import os
import threading
import urllib.parse
from dataclasses import dataclass, field
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .podresources import ALLOCATABLE_METHOD, MSG


@dataclass
class FakePod:
    uid: str
    namespace: str
    name: str
    node: str = "node-a"
    containers: dict = field(default_factory=dict)  # container name -> container id (no scheme)
    gpus: dict = field(default_factory=dict)        # container name -> [device ids]
    runtime: str = "containerd"
    phase: str = "Running"

    def to_json(self) -> dict:
        return {
            "metadata": {"uid": self.uid, "namespace": self.namespace, "name": self.name},
            "spec": {"nodeName": self.node, "containers": [{"name": c} for c in self.containers]},
            "status": {"phase": self.phase, "containerStatuses": [
                {"name": c, "containerID": f"{self.runtime}://{cid}" if cid else "", "ready": True}
                for c, cid in self.containers.items()]},
        }


class FakeKubelet:
    """PodResources gRPC server.  `pods` can be mutated between calls; `fail` injects
    UNAVAILABLE errors; `delay` injects slow responses (timeout tests)."""

    def __init__(self, socket_path: str, pods: list[FakePod] | None = None, resource: str = "amd.com/gpu",
                 node: str | None = None):
        self.socket_path = socket_path
        self.pods = list(pods or [])
        self.resource = resource
        self.node = node  # a real kubelet reports only its own node's pods
        self.fail = False
        self.delay = 0.0
        self.calls = 0
        self._server = None

    def _list(self, request, context):
        import time
        import grpc
        self.calls += 1
        if self.delay:
            time.sleep(self.delay)
        if self.fail:
            context.abort(grpc.StatusCode.UNAVAILABLE, "injected failure")
        resp = MSG["ListPodResourcesResponse"]()
        for p in self.pods:
            if self.node is not None and p.node != self.node:
                continue
            pr = resp.pod_resources.add()
            pr.name = p.name
            pr.namespace = p.namespace
            for cname in p.containers:
                c = pr.containers.add()
                c.name = cname
                ids = p.gpus.get(cname, [])
                if ids:
                    d = c.devices.add()
                    d.resource_name = self.resource
                    d.device_ids.extend(ids)
        return resp

    def _allocatable(self, request, context):
        resp = MSG["AllocatableResourcesResponse"]()
        return resp

    def start(self) -> "FakeKubelet":
        import grpc
        from concurrent import futures
        handlers = {
            "List": grpc.unary_unary_rpc_method_handler(
                self._list, request_deserializer=MSG["ListPodResourcesRequest"].FromString,
                response_serializer=MSG["ListPodResourcesResponse"].SerializeToString),
            "GetAllocatableResources": grpc.unary_unary_rpc_method_handler(
                self._allocatable, request_deserializer=MSG["AllocatableResourcesRequest"].FromString,
                response_serializer=MSG["AllocatableResourcesResponse"].SerializeToString),
        }
        assert ALLOCATABLE_METHOD.endswith("GetAllocatableResources")
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self._server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("v1.PodResourcesLister", handlers),))
        os.makedirs(os.path.dirname(self.socket_path), exist_ok=True)
        self._server.add_insecure_port("unix:" + self.socket_path)
        self._server.start()
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None


class FakeApiserver:
    """GET /api/v1/pods (list) and ?watch=1 (streaming events), node fieldSelector, bearer
    auth.  Mutate through add_pod / update_pod / delete_pod so watchers get events with
    increasing resourceVersions.  `fail_status` makes every request fail; `expire_before`
    answers watches from an older resourceVersion with 410 Gone (compacted history)."""

    def __init__(self, pods: list[FakePod] | None = None, token: str = "test-token"):
        self.pods = list(pods or [])
        self.token = token
        self.fail_status = 0
        self.requests: list[str] = []
        self.rv = 1
        self.expire_before = 0
        self._events: list[tuple[int, str, FakePod]] = []  # (rv, type, pod)
        self._cond = threading.Condition()
        self._stopping = False
        self._httpd = None
        self._thread = None

    # --- mutations (emit watch events) ---
    def _emit(self, typ: str, pod: FakePod) -> None:
        with self._cond:
            self.rv += 1
            self._events.append((self.rv, typ, pod))
            self._cond.notify_all()

    def add_pod(self, pod: FakePod) -> None:
        self.pods.append(pod)
        self._emit("ADDED", pod)

    def update_pod(self, pod: FakePod) -> None:
        self.pods = [pod if p.uid == pod.uid else p for p in self.pods]
        self._emit("MODIFIED", pod)

    def delete_pod(self, uid: str) -> None:
        gone = [p for p in self.pods if p.uid == uid]
        self.pods = [p for p in self.pods if p.uid != uid]
        for p in gone:
            self._emit("DELETED", p)

    def bookmark(self) -> None:
        with self._cond:
            self.rv += 1
            self._events.append((self.rv, "BOOKMARK", None))
            self._cond.notify_all()

    def _handler(self):
        fake = self

        def obj_json(pod: FakePod, rv: int) -> dict:
            o = pod.to_json()
            o["metadata"]["resourceVersion"] = str(rv)
            return o

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                fake.requests.append(self.path)
                if fake.fail_status:
                    self.send_response(fake.fail_status)
                    self.end_headers()
                    return
                if fake.token and self.headers.get("Authorization") != f"Bearer {fake.token}":
                    self.send_response(401)
                    self.end_headers()
                    return
                url = urllib.parse.urlparse(self.path)
                if url.path != "/api/v1/pods":
                    self.send_response(404)
                    self.end_headers()
                    return
                q = urllib.parse.parse_qs(url.query)
                node = None
                for sel in q.get("fieldSelector", []):
                    for term in sel.split(","):
                        k, _, v = term.partition("=")
                        if k == "spec.nodeName":
                            node = v
                if q.get("watch", ["0"])[0] in ("1", "true"):
                    return self._watch(q, node)
                items = [obj_json(p, fake.rv) for p in fake.pods if node is None or p.node == node]
                body = json.dumps({"kind": "PodList", "apiVersion": "v1",
                                   "metadata": {"resourceVersion": str(fake.rv)}, "items": items}).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _watch(self, q, node):
                import time
                since = int(q.get("resourceVersion", ["0"])[0] or 0)
                deadline = time.monotonic() + float(q.get("timeoutSeconds", ["5"])[0])
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.end_headers()  # HTTP/1.0: the stream ends when the connection closes
                if since < fake.expire_before:
                    ev = {"type": "ERROR", "object": {"kind": "Status", "code": 410, "reason": "Expired",
                                                      "message": "too old resource version"}}
                    self.wfile.write((json.dumps(ev) + "\n").encode())
                    return
                sent = since
                try:
                    while time.monotonic() < deadline and not fake._stopping and not fake.fail_status:
                        with fake._cond:
                            pending = [e for e in fake._events if e[0] > sent]
                            if not pending:
                                fake._cond.wait(0.05)
                                continue
                        for rv, typ, pod in pending:
                            sent = rv
                            if typ == "BOOKMARK":
                                ev = {"type": typ, "object": {"kind": "Pod", "metadata": {"resourceVersion": str(rv)}}}
                            elif node is not None and pod.node != node:
                                continue
                            else:
                                ev = {"type": typ, "object": obj_json(pod, rv)}
                            self.wfile.write((json.dumps(ev) + "\n").encode())
                            self.wfile.flush()
                except (BrokenPipeError, ConnectionResetError):
                    pass

        return H

    def start(self) -> "FakeApiserver":
        self._httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self._httpd.daemon_threads = True
        self._httpd.block_on_close = False
        self._thread = threading.Thread(target=self._httpd.serve_forever, daemon=True)
        self._thread.start()
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self._httpd.server_address[1]}"

    def stop(self) -> None:
        if self._httpd is not None:
            with self._cond:
                self._stopping = True  # open watch streams end
                self._cond.notify_all()
            self._httpd.shutdown()
            self._httpd.server_close()
            self._httpd = None
