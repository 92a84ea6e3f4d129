"""Deploy artefacts are consistent with the code: manifests parse, the DaemonSet's args are
accepted by the exporter's own CLI parser, the host mounts the design needs are present,
RBAC is read-only (the reference needed pods/exec), and every Helm value referenced by a
template exists in values.yaml."""
import os
import re

import pytest
import yaml

from kubernetes_gpu_exporter_amd.config import load_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K8S = os.path.join(ROOT, "deploy", "kubernetes")


def docs(name):
    with open(os.path.join(K8S, name)) as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


def test_manifests_parse():
    for f in os.listdir(K8S):
        assert docs(f), f


def test_daemonset_contract():
    (ds,) = docs("daemonset.yaml")
    spec = ds["spec"]["template"]["spec"]
    assert spec["hostPID"] is True  # KFD reports host PIDs
    c = spec["containers"][0]
    cfg = load_config(c["args"], env={"NODE_NAME": "n1"})
    assert cfg.backend == "amdsmi" and cfg.enable_counters and cfg.enable_rccl and cfg.listen == ":8000"
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert {"/sys", "/dev/kfd", "/dev/dri", "/var/lib/kubelet/pod-resources", "/var/log/pods"} <= mounts
    assert cfg.rccl_dir in mounts
    assert any(e["name"] == "NODE_NAME" for e in c["env"])
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"


def test_rbac_is_read_only():
    for d in docs("rbac.yaml"):
        if d["kind"] == "ClusterRole":
            for rule in d["rules"]:
                assert set(rule["verbs"]) <= {"get", "list", "watch"}
                assert "pods/exec" not in rule["resources"]


def test_helm_values_referenced_exist():
    chart = os.path.join(ROOT, "deploy", "helm", "gpuexp")
    with open(os.path.join(chart, "values.yaml")) as fh:
        values = yaml.safe_load(fh)
    refs = set()
    for f in os.listdir(os.path.join(chart, "templates")):
        with open(os.path.join(chart, "templates", f)) as fh:
            refs |= set(re.findall(r"\.Values\.([A-Za-z0-9_.]+)", fh.read()))
    assert refs
    for r in refs:
        node = values
        for part in r.split("."):
            assert isinstance(node, dict) and part in node, f"values.yaml lacks {r}"
            node = node[part]


def test_synthetic_workloads_use_known_models():
    from kubernetes_gpu_exporter_amd.models import WORKLOADS
    for d in docs("synthetic-workloads.yaml"):
        spec = d["spec"]["template"]["spec"] if d["kind"] == "Deployment" else d["spec"]
        cmd = spec["containers"][0]["command"]
        i = cmd.index("kubernetes_gpu_exporter_amd.models")
        assert cmd[i + 1] in WORKLOADS
        assert spec["containers"][0]["resources"]["limits"]["amd.com/gpu"] >= 1


def test_rules_reference_exported_metrics():
    """Every metric a recording/alert rule uses is one the exporter emits (docs/METRICS.md
    is generated from the engine)."""
    import re
    with open(os.path.join(os.path.dirname(K8S), "..", "docs", "METRICS.md")) as fh:
        known = set(re.findall(r"^\| `([a-z_:]+)` \|", fh.read(), re.M))
    assert "amd_gpu_up" in known
    used = set()
    for d in docs("rules.yaml"):
        for g in d["spec"]["groups"]:
            for rule in g["rules"]:
                for name in re.findall(r"\b((?:amd|gpuexp|pod_gpu|docker_gpu)_[a-z0-9_]+)", rule["expr"]):
                    used.add(re.sub(r"_(bucket|sum|count)$", "", name))
    assert used and used <= known, used - known


def test_grafana_dashboard_uses_exported_metrics():
    import json
    import re
    root = os.path.dirname(K8S)
    with open(os.path.join(root, "..", "docs", "METRICS.md")) as fh:
        known = set(re.findall(r"^\| `([a-z_:]+)` \|", fh.read(), re.M))
    with open(os.path.join(root, "grafana", "gpuexp-dashboard.json")) as fh:
        dash = json.load(fh)
    used = set()
    for p in dash["panels"]:
        for t in p["targets"]:
            for name in re.findall(r"\b((?:amd|gpuexp|pod_gpu|docker_gpu)_[a-z0-9_]+)", t["expr"]):
                used.add(re.sub(r"_(bucket|sum|count)$", "", name))
    for v in dash["templating"]["list"]:
        for name in re.findall(r"\b(amd_[a-z0-9_]+)", v.get("query", "")):
            used.add(name)
    assert len(dash["panels"]) >= 10 and used <= known, used - known


def test_memory_sized_for_one_queue_per_gpu():
    """Every GPU that gets the exporter's queue pins 346 MiB on MI355X
    (profiles/r02/queue_memory.txt): the static DaemonSet requests it for 8 GPUs, the Helm
    chart computes it from queueDevices / gpusPerNode."""
    (ds,) = docs("daemonset.yaml")
    c = ds["spec"]["template"]["spec"]["containers"][0]

    def mib(q):
        return int(q[:-2]) * (1024 if q.endswith("Gi") else 1)
    assert mib(c["resources"]["requests"]["memory"]) >= 40 + 8 * 346
    assert mib(c["resources"]["limits"]["memory"]) >= mib(c["resources"]["requests"]["memory"])
    chart = os.path.join(ROOT, "deploy", "helm", "gpuexp")
    with open(os.path.join(chart, "values.yaml")) as fh:
        values = yaml.safe_load(fh)
    assert values["memoryPerQueueGpuMi"] >= 346 and values["gpusPerNode"] == 8
    with open(os.path.join(chart, "templates", "daemonset.yaml")) as fh:
        tpl = fh.read()
    assert "mul $queueGpus .Values.memoryPerQueueGpuMi" in tpl and "--queue-devices=" in tpl
    cfg = load_config(["--queue-devices", "0,0000:72:00.0"], env={})
    assert cfg.queue_devices == ["0", "0000:72:00.0"]


def _hostpaths(spec):
    return {v["name"]: v["hostPath"] for v in spec.get("volumes", []) if "hostPath" in v}


def test_workload_hostpaths_are_created_by_the_daemonset():
    """Every hostPath a workload example mounts exists once the exporter DaemonSet ran on the
    node: it is a DaemonSet hostPath volume of type DirectoryOrCreate.  (Round 3 shipped a
    workload mounting /opt/gpuexp/lib with type Directory that nothing created.)"""
    (ds,) = docs("daemonset.yaml")
    ds_spec = ds["spec"]["template"]["spec"]
    created = {hp["path"] for hp in _hostpaths(ds_spec).values() if hp.get("type") == "DirectoryOrCreate"}
    checked = 0
    for f in ("example-workload.yaml", "synthetic-workloads.yaml"):
        for d in docs(f):
            spec = d["spec"]["template"]["spec"] if d["kind"] == "Deployment" else d["spec"]
            for name, hp in _hostpaths(spec).items():
                assert hp["path"] in created, (f, name, hp)
                checked += 1
    assert checked >= 3


def test_rccl_tracer_is_installed_where_workloads_load_it():
    """The init container installs libgpuexp_rccl_tracer.so into the host directory the
    example workload mounts, and the workload's ROCP_TOOL_LIBRARIES names that file."""
    from kubernetes_gpu_exporter_amd.utils.install_tracer import TRACER
    (ds,) = docs("daemonset.yaml")
    ds_spec = ds["spec"]["template"]["spec"]
    (init,) = [c for c in ds_spec["initContainers"] if c["name"] == "install-rccl-tracer"]
    assert init["command"][:3] == ["python3", "-m", "kubernetes_gpu_exporter_amd.utils.install_tracer"]
    dest = init["command"][3]
    (m,) = [m for m in init["volumeMounts"] if m["mountPath"] == dest]
    host_dir = _hostpaths(ds_spec)[m["name"]]["path"]
    (pod,) = docs("example-workload.yaml")
    c = pod["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in c["env"]}
    tool = env["ROCP_TOOL_LIBRARIES"]
    mount_dir, fname = os.path.split(tool)
    assert fname == TRACER
    (wm,) = [m for m in c["volumeMounts"] if m["mountPath"] == mount_dir]
    assert wm.get("readOnly") is True
    assert _hostpaths(pod["spec"])[wm["name"]]["path"] == host_dir
    # the Helm chart does the same when rccl.installTracer is on
    chart = os.path.join(ROOT, "deploy", "helm", "gpuexp")
    with open(os.path.join(chart, "templates", "daemonset.yaml")) as fh:
        tpl = fh.read()
    assert "install-rccl-tracer" in tpl and "kubernetes_gpu_exporter_amd.utils.install_tracer" in tpl
    with open(os.path.join(chart, "values.yaml")) as fh:
        values = yaml.safe_load(fh)
    assert values["rccl"]["installTracer"] is True and values["rccl"]["tracerHostDir"] == host_dir


def test_memory_limits_cover_the_read_rescue_worst_case():
    """Worst case: every queue GPU's PMC reads rescued at once (a node-wide job holding every
    wave slot): 40 MiB + 8 x (346 MiB queues + 173 MiB rescue queue).  The static limit covers
    it, and so does the Helm limit for 1..8 queue GPUs."""
    (ds,) = docs("daemonset.yaml")
    c = ds["spec"]["template"]["spec"]["containers"][0]

    def mib(q):
        return int(q[:-2]) * (1024 if q.endswith("Gi") else 1)
    worst = lambda n: 40 + n * (346 + 173)  # noqa: E731
    assert mib(c["resources"]["limits"]["memory"]) >= worst(8)
    chart = os.path.join(ROOT, "deploy", "helm", "gpuexp")
    with open(os.path.join(chart, "values.yaml")) as fh:
        v = yaml.safe_load(fh)
    with open(os.path.join(chart, "templates", "daemonset.yaml")) as fh:
        tpl = fh.read()
    assert "mul $queueGpus .Values.memoryPerRescueQueueMi" in tpl
    assert "add $mem $rescue .Values.resources.memoryLimitHeadroomMi" in tpl
    for n in range(1, 9):
        limit = 100 + n * v["memoryPerQueueGpuMi"] + n * v["memoryPerRescueQueueMi"] + v["resources"]["memoryLimitHeadroomMi"]
        assert limit >= worst(n), (n, limit, worst(n))


def test_helm_args_accepted_by_the_cli():
    """The Helm DaemonSet's exporter args, rendered with the chart's default values (a minimal
    stand-in for `helm template`: `{{ .Values.x }}` and `{{ join "," .Values.x }}`), parse with
    the exporter's own CLI parser and give the chart's settings."""
    chart = os.path.join(ROOT, "deploy", "helm", "gpuexp")
    with open(os.path.join(chart, "values.yaml")) as fh:
        values = yaml.safe_load(fh)

    def value(path):
        node = values
        for part in path.split("."):
            node = node[part]
        return node

    def render(line):
        line = re.sub(r'\{\{\s*join\s+"([^"]*)"\s+\.Values\.([A-Za-z0-9_.]+)\s*\}\}',
                      lambda m: m.group(1).join(str(x) for x in value(m.group(2))), line)
        return re.sub(r"\{\{\s*\.Values\.([A-Za-z0-9_.]+)\s*\}\}",
                      lambda m: str(value(m.group(1))).lower() if isinstance(value(m.group(1)), bool)
                      else str(value(m.group(1))), line)

    with open(os.path.join(chart, "templates", "daemonset.yaml")) as fh:
        text = fh.read()
    args = [render(m.group(1)) for m in re.finditer(r"^\s+- (--[a-z-]+=.*)$", text, re.M)
            if "{{ if" not in m.group(1) and "{{- " not in m.group(1)]
    args = [a for a in args if "{{" not in a]  # (conditional args stay out of this check)
    assert any(a.startswith("--exposition=") for a in args), args
    cfg = load_config(args, env={"NODE_NAME": "n1"})
    assert cfg.exposition == values["exposition"]
    assert str(cfg.metrics_min_interval) == str(values["metricsMinInterval"])
    assert cfg.metrics_cpu_budget == values["metricsCpuBudget"]
    # the option is a percent of one core: the chart must give the engine the same fraction as
    # the exporter's own default (round 5 shipped 0.015 = 0.015 %, 100x too small, which pinned
    # every Helm install's gpu_metrics refresh at metrics_max_interval)
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.config import Config
    n = load()
    assert cfg.to_engine_config(n).metrics_cpu_budget == pytest.approx(Config().to_engine_config(n).metrics_cpu_budget)
    assert Config().to_engine_config(n).metrics_cpu_budget == pytest.approx(0.0075)
    assert n.EngineConfig().metrics_cpu_budget == pytest.approx(0.0075)  # the engine's own default agrees
    assert cfg.counters_cpu_budget == values["countersCpuBudget"]
    assert cfg.to_engine_config(n).counters_cpu_budget == pytest.approx(n.EngineConfig().counters_cpu_budget)
    assert cfg.series_profile == values["seriesProfile"] and cfg.enable_counters == values["counters"]
