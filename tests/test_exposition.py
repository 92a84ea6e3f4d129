"""Exposition layer: value formatting, escaping, family ordering, stale-series GC,
histograms — checked against an independent strict parser."""
import math
import os

import pytest

from kubernetes_gpu_exporter_amd.utils import promtext


def test_format_value(native):
    f = native.format_value
    assert f(0.0) == "0"
    assert f(42.0) == "42"
    assert f(-7.0) == "-7"
    assert f(309220868096.0) == "309220868096"
    assert f(0.5) == "0.5"
    assert float(f(1 / 3)) == 1 / 3  # shortest round-trip
    assert f(float("nan")) == "NaN"
    assert f(float("inf")) == "+Inf"
    assert f(float("-inf")) == "-Inf"
    assert float(f(1e300)) == 1e300
    assert float(f(2.0 ** 60)) == 2.0 ** 60


@pytest.mark.parametrize("raw,esc", [
    ('a"b', 'a\\"b'), ("a\\b", "a\\\\b"), ("a\nb", "a\\nb"), ("plain", "plain"), ("", ""),
])
def test_label_escaping(native, raw, esc):
    assert native.escape_label_value(raw) == esc


def test_render_roundtrip_and_order(native):
    t = native.SeriesTable()
    g = native.MetricType.gauge
    fz = t.add_family("zeta_metric", "last\\family\nhelp", g, ["a"])
    fa = t.add_family("alpha_metric", "first", g, ["gpu", "pod"])
    t.put(fa, ["10", "p"], 1.0, 1)
    t.put(fa, ["9", "p"], 2.0, 1)
    t.put(fa, ["2", 'we"ird\\pod\n'], 3.5, 1)
    t.put(fz, ["x"], float("nan"), 1)
    text = t.render(1)
    fams = promtext.parse(text)
    assert list(fams) == ["alpha_metric", "zeta_metric"]  # sorted by name
    assert fams["zeta_metric"].help == "last\\family\nhelp"
    gpus = [s[1]["gpu"] for s in fams["alpha_metric"].samples]
    assert gpus == ["2", "9", "10"]  # numeric-aware label order
    assert promtext.value(fams, "alpha_metric", gpu="2") == 3.5
    assert fams["alpha_metric"].samples[0][1]["pod"] == 'we"ird\\pod\n'
    assert math.isnan(promtext.value(fams, "zeta_metric", a="x"))


def test_stale_series_gc(native):
    """A series not set in a tick disappears (reference never Reset(): main.go:147-150)."""
    t = native.SeriesTable()
    f = t.add_family("m", "h", native.MetricType.gauge, ["pid"])
    t.put(f, ["1"], 1, 1)
    t.put(f, ["2"], 2, 1)
    assert t.live_series(1) == 2
    t.put(f, ["1"], 1, 2)
    text = t.render(2)
    assert 'pid="2"' not in text and 'pid="1"' in text
    t.render(3)  # nothing set at gen 3 -> family omitted entirely
    assert t.render(4) == ""


def test_family_without_live_series_is_omitted(native):
    t = native.SeriesTable()
    t.add_family("never_set", "h", native.MetricType.gauge, [])
    assert t.render(1) == ""


def test_histogram_render(native):
    t = native.SeriesTable()
    f = t.add_family("lat_seconds", "h", native.MetricType.histogram, ["stage"])
    for v in (0.5e-6, 3e-6, 3e-6, 1.0):
        t.observe(f, ["render"], v, 1, [1e-6, 5e-6, 1e-3])
    fams = promtext.parse(t.render(1))
    s = {(n, l.get("le")): v for n, l, v in fams["lat_seconds"].samples}
    assert s[("lat_seconds_bucket", "1e-06")] == 1
    assert s[("lat_seconds_bucket", "5e-06")] == 3
    assert s[("lat_seconds_bucket", "0.001")] == 3
    assert s[("lat_seconds_bucket", "+Inf")] == 4
    assert s[("lat_seconds_count", None)] == 4
    assert abs(s[("lat_seconds_sum", None)] - (0.5e-6 + 6e-6 + 1.0)) < 1e-12


def test_invalid_names_rejected(native):
    t = native.SeriesTable()
    with pytest.raises(Exception):
        t.add_family("1bad", "h", native.MetricType.gauge, [])
    with pytest.raises(Exception):
        t.add_family("ok", "h", native.MetricType.gauge, ["bad-label"])
    with pytest.raises(Exception):
        t.add_family("ok2", "h", native.MetricType.gauge, ["__reserved"])
    f = t.add_family("ok3", "h", native.MetricType.gauge, ["a"])
    with pytest.raises(Exception):
        t.put(f, ["x", "y"], 1, 1)  # arity mismatch


def test_gzip_roundtrip(native):
    import gzip
    data = b"amd_gpu_up{gpu=\"0\"} 1\n" * 1000
    assert gzip.decompress(native.gzip(data)) == data


@pytest.mark.parametrize("impl", ["default", "zlib"])
def test_gzip_implementations(impl):
    """libdeflate (when the node has it) and the zlib fallback both emit valid gzip for
    bodies of every size, at every level; GPUEXP_GZIP_IMPL=zlib forces the fallback."""
    import subprocess
    import sys
    code = (
        "import gzip, os, random\n"
        "from kubernetes_gpu_exporter_amd._native import load\n"
        "n = load()\n"
        "random.seed(1)\n"
        "for size in (0, 1, 100, 65536, 300000):\n"
        "    data = bytes(random.choice(b'amd_gpu {}=\"0123456789.\\n') for _ in range(size))\n"
        "    for level in (1, 6, 9):\n"
        "        assert gzip.decompress(n.gzip(data, level)) == data, (size, level)\n"
        "print(n.gzip_impl())\n")
    env = dict(os.environ)
    if impl == "zlib":
        env["GPUEXP_GZIP_IMPL"] = "zlib"
    else:
        env.pop("GPUEXP_GZIP_IMPL", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    used = r.stdout.strip()
    assert used == "zlib" if impl == "zlib" else used in ("libdeflate", "zlib")


def test_exposition_parses_with_prometheus_client(mock_engine):
    """An independent parser (the official Python client's text-format parser) accepts the
    full 8-GPU exposition, with processes, pods, histograms and escaped label values, and
    reads back the same families, types and sample values as ours."""
    from prometheus_client.parser import text_string_to_metric_families
    e = mock_engine(8, http=False, series_profile="full", enable_sentinel=True, enable_counters=True)
    uid = "12345678-1234-1234-1234-123456789abc"
    cg = ("/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod" + uid.replace("-", "_")
          + ".slice/cri-containerd-" + "a" * 64 + ".scope")
    e.mock_set_processes(0, [dict(pid=42, vram_bytes=3.0e9, cu_occupancy=64, name='we"ird\\comm')])
    e.set_pid_cgroup(42, cg)
    e.set_pods([dict(uid=uid, namespace="ns", name="pod-a", containers={"a" * 64: "main"})])
    for i in range(3):
        e.tick((i + 1) * 100_000_000)
    text = e.snapshot_text()
    ours = promtext.parse(text)
    theirs = {f.name: f for f in text_string_to_metric_families(text)}
    for name, fam in ours.items():
        # the official parser strips _total from counter family names
        tf = theirs.get(name) or theirs.get(name[:-6] if name.endswith("_total") else name)
        assert tf is not None, name
        assert tf.type == fam.type, (name, tf.type, fam.type)
        got = {(s.name, tuple(sorted(s.labels.items()))): s.value for s in tf.samples}
        for sname, lab, v in fam.samples:
            key = (sname, tuple(sorted((k, str(x)) for k, x in lab.items())))
            assert key in got, (name, key)
            assert got[key] == v or (math.isnan(v) and math.isnan(got[key])), (key, got[key], v)
    (comm,) = [s.labels["comm"] for s in theirs["amd_gpu_process_vram_bytes"].samples]
    assert comm == 'we"ird\\comm'
