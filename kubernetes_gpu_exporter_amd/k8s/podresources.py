"""kubelet PodResources v1 gRPC client (and the message classes used by the fake kubelet).

grpcio-tools is not available, so the `k8s.io/kubelet/pkg/apis/podresources/v1` messages
are declared programmatically with descriptor_pb2 — same field numbers as the upstream
api.proto, so the wire format is identical.  The ROCm k8s device plugin registers GPUs
under the resource `amd.com/gpu` with PCI BDFs as device IDs; both BDF and UUID keys are
accepted by the engine when matching devices to owners.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from .controlplane import Metadata, Source

LIST_METHOD = "/v1.PodResourcesLister/List"
ALLOCATABLE_METHOD = "/v1.PodResourcesLister/GetAllocatableResources"

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "gpuexp/podresources_v1.proto"
    fdp.package = "v1"
    fdp.syntax = "proto3"

    def msg(name, fields):
        m = fdp.message_type.add()
        m.name = name
        for num, fname, ftype, label, tname in fields:
            f = m.field.add()
            f.name = fname
            f.number = num
            f.type = ftype
            f.label = label
            if tname:
                f.type_name = tname

    REP, OPT = _F.LABEL_REPEATED, _F.LABEL_OPTIONAL
    S, I64, MSG = _F.TYPE_STRING, _F.TYPE_INT64, _F.TYPE_MESSAGE
    msg("ListPodResourcesRequest", [])
    msg("NUMANode", [(1, "ID", I64, OPT, None)])
    msg("TopologyInfo", [(1, "nodes", MSG, REP, ".v1.NUMANode")])
    msg("ContainerDevices", [(1, "resource_name", S, OPT, None), (2, "device_ids", S, REP, None),
                             (3, "topology", MSG, OPT, ".v1.TopologyInfo")])
    msg("ContainerMemory", [(1, "memory_type", S, OPT, None), (2, "size", _F.TYPE_UINT64, OPT, None),
                            (3, "topology", MSG, OPT, ".v1.TopologyInfo")])
    msg("ContainerResources", [(1, "name", S, OPT, None), (2, "devices", MSG, REP, ".v1.ContainerDevices"),
                               (3, "cpu_ids", I64, REP, None), (4, "memory", MSG, REP, ".v1.ContainerMemory")])
    msg("PodResources", [(1, "name", S, OPT, None), (2, "namespace", S, OPT, None),
                         (3, "containers", MSG, REP, ".v1.ContainerResources")])
    msg("ListPodResourcesResponse", [(1, "pod_resources", MSG, REP, ".v1.PodResources")])
    msg("AllocatableResourcesRequest", [])
    msg("AllocatableResourcesResponse", [(1, "devices", MSG, REP, ".v1.ContainerDevices"),
                                         (2, "cpu_ids", I64, REP, None),
                                         (3, "memory", MSG, REP, ".v1.ContainerMemory")])
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    out = {}
    for name in ("ListPodResourcesRequest", "ListPodResourcesResponse", "PodResources", "ContainerResources",
                 "ContainerDevices", "TopologyInfo", "NUMANode", "AllocatableResourcesRequest",
                 "AllocatableResourcesResponse"):
        out[name] = message_factory.GetMessageClass(pool.FindMessageTypeByName("v1." + name))
    return out


MSG = _build()
ListPodResourcesRequest = MSG["ListPodResourcesRequest"]
ListPodResourcesResponse = MSG["ListPodResourcesResponse"]


def resource_matches(name: str, patterns) -> bool:
    """Exact resource names or shell-style patterns ("amd.com/*px_nps*")."""
    import fnmatch
    return any(name == p or (any(ch in p for ch in "*?[") and fnmatch.fnmatchcase(name, p)) for p in patterns)


def owners_from_response(resp, resource_names) -> dict:
    """device_id -> {namespace, pod, container} for the GPU resources.

    Device ids are passed through as the device plugin reports them (lower-cased): a PCI
    BDF for a whole GPU, and in partition mode an id per logical GPU (the BDF for
    partition 0, the XCP platform device "amdgpu_xcp_<n>" / "amdgpu_xcp.<n>" for the
    others, or "<bdf>/<n>", a render node, "kfd:<gpu_id>", a UUID).  The engine matches
    them against each logical GPU's keys (device_owner_keys in csrc/gpuexp/device.h), so
    partitions of one socket given to different pods keep different owners."""
    owners = {}
    for pr in resp.pod_resources:
        for c in pr.containers:
            for d in c.devices:
                if not resource_matches(d.resource_name, resource_names):
                    continue
                for dev_id in d.device_ids:
                    owners[dev_id.lower()] = {"namespace": pr.namespace, "pod": pr.name, "container": c.name}
    return owners


class PodResourcesSource(Source):
    name = "podresources"

    def __init__(self, socket_path: str, resource_names=("amd.com/gpu",), timeout: float = 3.0):
        self.socket_path = socket_path
        self.resource_names = list(resource_names)
        self.timeout = timeout
        self._channel = None
        self._list = None

    def _stub(self):
        if self._list is None:
            import grpc
            self._channel = grpc.insecure_channel("unix://" + self.socket_path)
            self._list = self._channel.unary_unary(LIST_METHOD,
                                                   request_serializer=ListPodResourcesRequest.SerializeToString,
                                                   response_deserializer=ListPodResourcesResponse.FromString)
        return self._list

    def fetch(self) -> Metadata:
        try:
            resp = self._stub()(ListPodResourcesRequest(), timeout=self.timeout)
        except Exception:
            # reconnect next time (kubelet restarts recreate the socket)
            if self._channel is not None:
                self._channel.close()
            self._channel = self._list = None
            raise
        md = Metadata()
        md.owners = owners_from_response(resp, self.resource_names)
        return md

    def close(self) -> None:
        if self._channel is not None:
            self._channel.close()
