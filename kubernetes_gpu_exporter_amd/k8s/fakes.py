"""Fakes for the Kubernetes control plane (there is no cluster in CI or on the GPU box).

FakeKubelet    — PodResources v1 gRPC server on a unix socket (same wire format as the
                 kubelet: `/v1.PodResourcesLister/List`).
FakeApiserver  — HTTP server for GET /api/v1/pods with fieldSelector=spec.nodeName and
                 bearer-token auth, returning PodList JSON shaped like the real thing.
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
    def __init__(self, pods: list[FakePod] | None = None, token: str = "test-token"):
        self.pods = list(pods or [])
        self.token = token
        self.fail_status = 0
        self.requests: list[str] = []
        self._httpd = None
        self._thread = None

    def _handler(self):
        fake = self

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
                items = [p.to_json() for p in fake.pods if node is None or p.node == node]
                body = json.dumps({"kind": "PodList", "apiVersion": "v1",
                                   "metadata": {"resourceVersion": "1"}, "items": items}).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        return H

    def start(self) -> "FakeApiserver":
        self._httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self._thread = threading.Thread(target=self._httpd.serve_forever, daemon=True)
        self._thread.start()
        return self

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self._httpd.server_address[1]}"

    def stop(self) -> None:
        if self._httpd is not None:
            self._httpd.shutdown()
            self._httpd.server_close()
            self._httpd = None
