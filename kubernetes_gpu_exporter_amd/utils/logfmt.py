"""logfmt for the Python control plane, byte-compatible with the C++ core's log lines
(csrc/gpuexp/common.cc log_msg): `ts=<unix s.ms> level=<debug|info|warn|error>
component=<name> msg="<escaped>"`, one record per line on stderr, so both halves of the
exporter interleave into one parseable stream.  `log_format: json` switches both halves to
one JSON object per line with the same keys (ts, level, component, msg).  The reference logged unstructured
fmt.Printf text every cycle (/root/reference/main.go:81, 89, 104, 108)."""
from __future__ import annotations

import json
import logging

_LEVELS = {logging.DEBUG: "debug", logging.INFO: "info", logging.WARNING: "warn", logging.ERROR: "error",
           logging.CRITICAL: "error"}


def escape(v: str) -> str:
    return v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", " ")


class LogfmtFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        msg = record.getMessage()
        if record.exc_info:
            msg += " " + self.formatException(record.exc_info)
        level = _LEVELS.get(record.levelno, "info")
        component = record.name[len("gpuexp."):] if record.name.startswith("gpuexp.") else record.name
        return f'ts={record.created:.3f} level={level} component={component} msg="{escape(msg)}"'


class JsonFormatter(LogfmtFormatter):
    def format(self, record: logging.LogRecord) -> str:
        msg = record.getMessage()
        if record.exc_info:
            msg += " " + self.formatException(record.exc_info)
        component = record.name[len("gpuexp."):] if record.name.startswith("gpuexp.") else record.name
        return json.dumps({"ts": round(record.created, 3), "level": _LEVELS.get(record.levelno, "info"),
                           "component": component, "msg": msg.replace("\n", " ")})


def setup(level: str, fmt: str = "logfmt") -> None:
    """Root logging to stderr at the exporter's --log-level, as logfmt or JSON lines."""
    h = logging.StreamHandler()
    h.setFormatter(JsonFormatter() if fmt == "json" else LogfmtFormatter())
    root = logging.getLogger()
    for old in list(root.handlers):
        root.removeHandler(old)
    root.addHandler(h)
    root.setLevel({"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING, "error": logging.ERROR,
                   "off": logging.CRITICAL + 10}[level])
