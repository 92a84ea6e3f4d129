#!/usr/bin/env python3
"""GPU-box probe: how much of the exposition changes from one tick to the next (what an
incremental per-family gzip could reuse).  Runs the amdsmi engine (full profile, sentinel,
counters) with manual ticks 100 ms apart and compares consecutive snapshots family by
family.  Usage: python tools/probe_body_churn.py [ticks]"""
import json
import os
import sys
import time
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def families(text: str) -> dict:
    out, cur, buf = {}, None, []
    for line in text.splitlines(keepends=True):
        if line.startswith("# HELP "):
            if cur is not None:
                out[cur] = "".join(buf)
            cur, buf = line.split()[2], []
        buf.append(line)
    if cur is not None:
        out[cur] = "".join(buf)
    return out


def main() -> int:
    n_ticks = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch  # noqa: F401  (HIP runtime first, as the exporter's sentinel expects)
    from kubernetes_gpu_exporter_amd._native import load
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0
    c.serve_http = False
    c.series_profile = "full"
    c.enable_sentinel = True
    c.enable_counters = True
    e = n.Engine(c)
    e.start()
    prev = None
    changed = total = 0
    per_family: dict = {}
    for _ in range(n_ticks):
        e.tick()
        time.sleep(0.1)
        fams = families(e.snapshot_text())
        if prev is not None:
            for k, v in fams.items():
                total += len(v)
                if prev.get(k) != v:
                    changed += len(v)
                    per_family[k] = per_family.get(k, 0) + 1
        prev = fams
    body = "".join(prev.values()).encode()
    e.stop()
    print("RESULT " + json.dumps({
        "body_bytes": len(body), "gzip1_bytes": len(zlib.compress(body, 1)),
        "changed_byte_fraction": round(changed / max(1, total), 3),
        "families": len(prev), "families_changing_every_tick": sorted(k for k, v in per_family.items()
                                                                     if v == n_ticks - 1),
        "families_never_changing": sorted(k for k in prev if k not in per_family)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
