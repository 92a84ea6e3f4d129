"""Decoder for the delimited protobuf exposition (io.prometheus.client.MetricFamily).

client_golang's promhttp (the reference's handler, /root/reference/main.go:70) serves this
format when a scraper's Accept header negotiates it; the exporter does the same.  The
metrics.proto messages are declared programmatically (no protoc here) with the upstream
field numbers, so this parses real Prometheus wire data too.  Used by tests and tools.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf.internal.decoder import _DecodeVarint32

ACCEPT = ("application/vnd.google.protobuf;proto=io.prometheus.client.MetricFamily;encoding=delimited;q=0.7,"
          "text/plain;version=0.0.4;q=0.3,*/*;q=0.1")
TYPES = {0: "counter", 1: "gauge", 2: "summary", 3: "untyped", 4: "histogram", 5: "gaugehistogram"}

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "gpuexp/metrics.proto"
    fdp.package = "io.prometheus.client"
    fdp.syntax = "proto2"
    en = fdp.enum_type.add()
    en.name = "MetricType"
    for num, nm in TYPES.items():
        v = en.value.add()
        v.name = nm.upper()
        v.number = num

    def msg(name, fields):
        m = fdp.message_type.add()
        m.name = name
        for num, fname, ftype, label, tname in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = fname, num, ftype, label
            if tname:
                f.type_name = tname

    OPT, REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    S, D, U64, MSG, ENUM, I64 = _F.TYPE_STRING, _F.TYPE_DOUBLE, _F.TYPE_UINT64, _F.TYPE_MESSAGE, _F.TYPE_ENUM, _F.TYPE_INT64
    P = ".io.prometheus.client."
    msg("LabelPair", [(1, "name", S, OPT, None), (2, "value", S, OPT, None)])
    msg("Gauge", [(1, "value", D, OPT, None)])
    msg("Counter", [(1, "value", D, OPT, None)])
    msg("Untyped", [(1, "value", D, OPT, None)])
    msg("Bucket", [(1, "cumulative_count", U64, OPT, None), (2, "upper_bound", D, OPT, None)])
    msg("Histogram", [(1, "sample_count", U64, OPT, None), (2, "sample_sum", D, OPT, None),
                      (3, "bucket", MSG, REP, P + "Bucket")])
    msg("Metric", [(1, "label", MSG, REP, P + "LabelPair"), (2, "gauge", MSG, OPT, P + "Gauge"),
                   (3, "counter", MSG, OPT, P + "Counter"), (5, "untyped", MSG, OPT, P + "Untyped"),
                   (6, "timestamp_ms", I64, OPT, None), (7, "histogram", MSG, OPT, P + "Histogram")])
    msg("MetricFamily", [(1, "name", S, OPT, None), (2, "help", S, OPT, None), (3, "type", ENUM, OPT, P + "MetricType"),
                         (4, "metric", MSG, REP, P + "Metric")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("io.prometheus.client.MetricFamily"))


MetricFamily = _build()


def parse_delimited(data: bytes) -> list:
    """Returns [MetricFamily, ...] from a varint-length-delimited stream."""
    out, pos = [], 0
    while pos < len(data):
        n, pos = _DecodeVarint32(data, pos)
        mf = MetricFamily()
        mf.ParseFromString(data[pos:pos + n])
        pos += n
        out.append(mf)
    return out


def to_samples(families: list) -> dict:
    """{family: (type, help, [(labels dict, value)])} with histograms flattened to their
    text-format samples (_bucket incl. +Inf, _sum, _count) for comparison with promtext."""
    res = {}
    for mf in families:
        typ = TYPES[mf.type]
        rows = []
        for m in mf.metric:
            labels = {lp.name: lp.value for lp in m.label}
            if typ == "histogram":
                h = m.histogram
                for b in h.bucket:
                    rows.append((f"{mf.name}_bucket", dict(labels, le=b.upper_bound), float(b.cumulative_count)))
                rows.append((f"{mf.name}_bucket", dict(labels, le=float("inf")), float(h.sample_count)))
                rows.append((f"{mf.name}_sum", labels, h.sample_sum))
                rows.append((f"{mf.name}_count", labels, float(h.sample_count)))
            elif typ == "counter":
                rows.append((mf.name, labels, m.counter.value))
            else:
                rows.append((mf.name, labels, m.gauge.value))
        res[mf.name] = (typ, mf.help, rows)
    return res


def to_promtext(families: list) -> dict:
    """Same shape as utils.promtext.parse(): {name: Family(name, help, type, samples)}."""
    from .promtext import Family
    out = {}
    for name, (typ, helptext, rows) in to_samples(families).items():
        fam = Family(name, helptext, typ)
        for sname, labels, v in rows:
            lab = {k: (("+Inf" if v2 == float("inf") else repr(float(v2))) if k == "le" else v2)
                   for k, v2 in labels.items()}
            fam.samples.append((sname, lab, v))
        out[name] = fam
    return out
