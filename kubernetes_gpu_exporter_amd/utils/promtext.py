"""Strict parser for Prometheus text exposition 0.0.4 (used by tests and the bench to
validate every byte the exporter serves, independently of the C++ renderer)."""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field

_NAME = re.compile(r"[a-zA-Z_:][a-zA-Z0-9_:]*")
_LABEL = re.compile(r"[a-zA-Z_][a-zA-Z0-9_]*")


@dataclass
class Family:
    name: str
    help: str = ""
    type: str = "untyped"
    samples: list = field(default_factory=list)  # (sample_name, labels dict, value)


class ParseError(ValueError):
    pass


def _unescape(s: str, label: bool) -> str:
    out = []
    i = 0
    while i < len(s):
        c = s[i]
        if c == "\\" and i + 1 < len(s):
            n = s[i + 1]
            if n == "n":
                out.append("\n")
            elif n == "\\":
                out.append("\\")
            elif n == '"' and label:
                out.append('"')
            else:
                out.append("\\" + n)
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


def _parse_value(tok: str) -> float:
    if tok in ("+Inf", "Inf"):
        return math.inf
    if tok == "-Inf":
        return -math.inf
    if tok == "NaN":
        return math.nan
    return float(tok)


def _parse_labels(s: str, pos: int, line: str) -> tuple[dict, int]:
    labels = {}
    assert s[pos] == "{"
    pos += 1
    while True:
        if s[pos] == "}":
            return labels, pos + 1
        m = _LABEL.match(s, pos)
        if not m:
            raise ParseError(f"bad label name in: {line}")
        name = m.group(0)
        pos = m.end()
        if s[pos:pos + 2] != '="':
            raise ParseError(f"expected =\" in: {line}")
        pos += 2
        buf = []
        while True:
            if pos >= len(s):
                raise ParseError(f"unterminated label value: {line}")
            c = s[pos]
            if c == "\\":
                buf.append(s[pos:pos + 2])
                pos += 2
                continue
            if c == '"':
                pos += 1
                break
            if c == "\n":
                raise ParseError("raw newline in label value")
            buf.append(c)
            pos += 1
        if name in labels:
            raise ParseError(f"duplicate label {name}: {line}")
        labels[name] = _unescape("".join(buf), True)
        if s[pos] == ",":
            pos += 1
        elif s[pos] != "}":
            raise ParseError(f"expected , or }} in: {line}")


def parse(text: str) -> dict[str, Family]:
    fams: dict[str, Family] = {}
    seen_series = set()
    cur: Family | None = None
    if text and not text.endswith("\n"):
        raise ParseError("exposition must end with a newline")
    for line in text.split("\n"):
        if not line:
            continue
        if line.startswith("# HELP "):
            rest = line[7:]
            name, _, h = rest.partition(" ")
            cur = fams.setdefault(name, Family(name))
            cur.help = _unescape(h, False)
            continue
        if line.startswith("# TYPE "):
            name, _, t = line[7:].partition(" ")
            if t not in ("gauge", "counter", "histogram", "summary", "untyped"):
                raise ParseError(f"bad type {t}")
            cur = fams.setdefault(name, Family(name))
            if cur.samples:
                raise ParseError(f"TYPE after samples for {name}")
            cur.type = t
            continue
        if line.startswith("#"):
            continue
        m = _NAME.match(line)
        if not m:
            raise ParseError(f"bad sample line: {line}")
        sname = m.group(0)
        pos = m.end()
        labels = {}
        if pos < len(line) and line[pos] == "{":
            labels, pos = _parse_labels(line, pos, line)
        if pos >= len(line) or line[pos] != " ":
            raise ParseError(f"expected space before value: {line}")
        # any run of blanks around the value (the compiled exposition right-aligns values)
        toks = line[pos + 1:].split()
        if not toks or len(toks) > 2:
            raise ParseError(f"expected value [timestamp]: {line}")
        value = _parse_value(toks[0])
        base = sname
        for suf in ("_bucket", "_sum", "_count"):
            if sname.endswith(suf) and sname[: -len(suf)] in fams and fams[sname[: -len(suf)]].type == "histogram":
                base = sname[: -len(suf)]
        fam = fams.get(base)
        if fam is None:
            fam = fams.setdefault(base, Family(base))
        key = (sname, tuple(sorted(labels.items())))
        if key in seen_series:
            raise ParseError(f"duplicate series: {line}")
        seen_series.add(key)
        fam.samples.append((sname, labels, value))
    return fams


def samples(fams: dict[str, Family], name: str) -> list:
    f = fams.get(name)
    return [] if f is None else f.samples


def value(fams: dict[str, Family], name: str, **labels) -> float:
    for sname, lab, v in samples(fams, name):
        if sname == name and all(lab.get(k) == str(val) for k, val in labels.items()):
            return v
    raise KeyError(f"{name}{labels}")
