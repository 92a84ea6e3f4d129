"""Loader for the in-tree native module (`_gpuexp`, built by build_native.py).

The native core is mandatory: there is no pure-Python fallback for the sampler, the
exposition renderer or the HTTP server, so a missing extension fails loudly instead of
silently degrading (the round-end GPU check records which .so files were loaded).
"""
from __future__ import annotations

import importlib
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
_mod = None


def load():
    """Imports and returns the `_gpuexp` extension module (builds it if GPUEXP_AUTOBUILD=1)."""
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("kubernetes_gpu_exporter_amd._gpuexp")
    except ImportError as e:
        if os.environ.get("GPUEXP_AUTOBUILD") == "1":
            import subprocess
            import sys
            subprocess.check_call([sys.executable, str(PKG_DIR.parent / "build_native.py")])
            _mod = importlib.import_module("kubernetes_gpu_exporter_amd._gpuexp")
        else:
            raise ImportError(
                "native module _gpuexp is not built; run `python build_native.py` "
                f"(or set GPUEXP_AUTOBUILD=1): {e}") from e
    return _mod


def rocprof_plugin_path(kind: str = "aqlpmc") -> str:
    """Counter plugin: "aqlpmc" (default, aqlprofile on an owned queue) or "rocprof"
    (rocprofiler-sdk device counting; costs a spinning runtime thread, see rocprof_plugin.cc)."""
    return str(PKG_DIR / ("_gpuexp_aqlpmc.so" if kind == "aqlpmc" else "_gpuexp_rocprof.so"))


def rccl_tracer_path() -> str:
    return str(PKG_DIR / "libgpuexp_rccl_tracer.so")
