"""Docs generated from code stay in sync with it."""
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_metrics_reference_is_current(native):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_metrics_doc.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, "docs/METRICS.md is stale: run python tools/gen_metrics_doc.py\n" + r.stderr
