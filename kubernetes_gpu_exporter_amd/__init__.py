"""MI355X-native per-pod GPU telemetry exporter.

Same capabilities as dorkamotorka/kubernetes-gpu-exporter (a single Go main() that joins
NVML compute processes to Kubernetes pods and exposes `pod_gpu_memory_usage` and
`docker_gpu_memory_perc_usage{pid,pod}` on :8000/metrics — /root/reference/main.go),
re-designed MI355X-first: a C++ data plane (amdsmi / KFD sysfs / raw gpu_metrics /
rocprofiler-sdk / HIP sentinel kernel) serving pre-rendered snapshots, and a Python
control plane (kubelet PodResources, node-scoped pod metadata).

Subpackages:
  models/    metric-family schema and series profiles (the /metrics contract)
  ops/       HIP kernels: sentinel + MFMA GEMM workload wrappers
  parallel/  RCCL collective traffic generators (DP/TP/PP/SP/EP/CP/Ulysses) + launchers
  k8s/       PodResources gRPC client, pod metadata sources, control plane, fakes
  utils/     exposition parser, process CPU accounting, fake host roots, scraping
"""
__version__ = "0.1.0"

__all__ = ["__version__", "Config", "Exporter", "load_config"]


def __getattr__(name):
    if name == "Config":
        from .config import Config
        return Config
    if name == "load_config":
        from .config import load_config
        return load_config
    if name == "Exporter":
        from .exporter import Exporter
        return Exporter
    raise AttributeError(name)
