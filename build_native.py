#!/usr/bin/env python3
"""Builds the native parts of the exporter in-tree for gfx950.

Outputs (all inside kubernetes_gpu_exporter_amd/, so they travel with the repo):
  _gpuexp<EXT_SUFFIX>        pybind11 module: C++ telemetry core + HIP sentinel + MFMA GEMM
  _gpuexp_aqlpmc.so          device PMC plugin: aqlprofile PM4 on an owned HSA queue (default)
  _gpuexp_rocprof.so         rocprofiler-sdk device-counting plugin (alternative counter backend)
  libgpuexp_rccl_tracer.so   rocprofiler-sdk RCCL API-tracing tool (ROCP_TOOL_LIBRARIES)

C++ (.cc) compiles with g++, HIP (.hip) with hipcc --offload-arch=gfx950; the module is
linked with hipcc.  Incremental: an object is rebuilt when its source or any header under
csrc/ is newer.  Usage: python build_native.py [--force] [-j N] [--sanitize address]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
PKG = ROOT / "kubernetes_gpu_exporter_amd"
BUILD = ROOT / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("GPUEXP_OFFLOAD_ARCH", "gfx950")

CORE_CC = [
    "gpuexp/common.cc", "gpuexp/exposition.cc", "gpuexp/deflate_tmpl.cc", "gpuexp/gzip.cc", "gpuexp/http.cc",
    "gpuexp/gpu_metrics.cc", "gpuexp/backend_mock.cc", "gpuexp/backend_sysfs.cc",
    "gpuexp/backend_amdsmi.cc", "gpuexp/procs.cc", "gpuexp/ras.cc", "gpuexp/kfd_events.cc", "gpuexp/engine.cc", "gpuexp/engine_device.cc", "gpuexp/engine_procs.cc",
    "gpuexp/engine_pods.cc", "gpuexp/engine_rccl.cc", "gpuexp/engine_kfd_events.cc", "gpuexp/engine_self.cc",
    "gpuexp/engine_state.cc", "gpuexp/fake_sources.cc",
    "gpuexp/optional_sources.cc", "gpuexp/client.cc", "gpuexp/pmc_rounds.cc", "gpuexp/pmc_harness.cc",
    "gpuexp/pmc_agents.cc", "bindings.cc",
]
SENTINEL_HIP = ["gpuexp/sentinel.hip"]
SENTINEL_HSACO = "gpuexp/sentinel_hsaco.hip"  # device-only code object for raw AQL dispatch
CALIB_HSACO = "kernels/calib_hsaco.hip"       # PMC calibration workloads, dispatched on the PMC queue
KERNELS_HIP = ["kernels/gemm_bf16.hip", "kernels/probe_kernels.hip", "kernels/kernels_bindings.hip"]
ROCPROF_CC = ["gpuexp/rocprof_plugin.cc"]
AQLPMC_CC = ["gpuexp/aql_pmc.cc"]
TRACER_CC = ["gpuexp/rccl_tracer.cc"]


def _pybind_include() -> str:
    import pybind11
    return pybind11.get_include()


def _hdr_mtime() -> float:
    return max((p.stat().st_mtime for p in CSRC.rglob("*.h")), default=0.0)


def _needs(obj: Path, src: Path, hdr_mtime: float, force: bool) -> bool:
    if force or not obj.exists():
        return True
    m = obj.stat().st_mtime
    return m < src.stat().st_mtime or m < hdr_mtime


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def _common_flags(sanitize: str | None) -> list[str]:
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O2", "-g1", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-parameter",
             f"-I{CSRC}", f"-I{ROCM / 'include'}", f"-I{_pybind_include()}", f"-I{py_inc}",
             "-D__HIP_PLATFORM_AMD__"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
    return flags


def compile_one(src_rel: str, hdr_mtime: float, force: bool, sanitize: str | None) -> Path:
    src = CSRC / src_rel
    obj = BUILD / (src_rel.replace("/", "__") + ".o")
    if not _needs(obj, src, hdr_mtime, force):
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    if src.suffix == ".hip":
        cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-x", "hip"] + _common_flags(None)
        if sanitize:
            # Host-side sanitizer only: GPU ASan is not available on this pool.
            cmd += ["-Xarch_host", f"-fsanitize={sanitize}", "-fno-gpu-sanitize"]
    else:
        cmd = ["g++"] + _common_flags(sanitize)
    cmd += ["-c", str(src), "-o", str(obj)]
    _run(cmd)
    return obj


def _ext(name: str) -> Path:
    return PKG / f"{name}{sysconfig.get_config_var('EXT_SUFFIX') or '.so'}"


def link_core(objs: list[Path], sanitize: str | None) -> Path:
    """The telemetry core links NO HIP runtime (see sentinel.hip's factory comment)."""
    out = _ext("_gpuexp")
    tmp = out.with_suffix(".tmp.so")
    cmd = ["g++", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
    cmd += [f"-L{ROCM / 'lib'}", "-lamd_smi", "-lz", "-ldl", "-lpthread", f"-Wl,-rpath,{ROCM / 'lib'}"]
    if sanitize:
        cmd += [f"-fsanitize={sanitize}"]
    _run(cmd)
    os.replace(tmp, out)
    return out


def link_hip(objs: list[Path], out: Path, libs: list[str]) -> Path:
    tmp = out.with_suffix(".tmp.so")
    _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] +
         [str(o) for o in objs] + [f"-L{ROCM / 'lib'}"] + libs + [f"-Wl,-rpath,{ROCM / 'lib'}"])
    os.replace(tmp, out)
    return out


def build_hsaco(src: str, out: Path, hdr_mtime: float, force: bool) -> Path:
    """A plain gfx950 code object (no host code, no offload bundle) for hsa_executable loading."""
    s = CSRC / src
    if not _needs(out, s, hdr_mtime, force):
        return out
    tmp = out.with_suffix(".tmp.hsaco")
    _run([str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "--cuda-device-only", "--no-gpu-bundle-output",
          "-O3", "-std=c++17", f"-I{CSRC}", "-o", str(tmp), str(s)])
    os.replace(tmp, out)
    return out


def link_plain(objs: list[Path], out: Path, libs: list[str]) -> Path:
    tmp = out.with_suffix(".tmp.so")
    _run(["g++", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs] +
         [f"-L{ROCM / 'lib'}"] + libs + [f"-Wl,-rpath,{ROCM / 'lib'}"])
    os.replace(tmp, out)
    return out


def build(force: bool = False, jobs: int = 8, sanitize: str | None = None, verbose: bool = True) -> dict:
    hdr = _hdr_mtime()
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = CORE_CC + SENTINEL_HIP + KERNELS_HIP
    extra = [s for s in ROCPROF_CC + AQLPMC_CC + TRACER_CC if (CSRC / s).exists()]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {s: ex.submit(compile_one, s, hdr, force, sanitize) for s in srcs + extra}
        objs = {s: f.result() for s, f in futs.items()}
    outputs = {
        "module": str(link_core([objs[s] for s in CORE_CC], sanitize)),
        "sentinel": str(link_hip([objs[s] for s in SENTINEL_HIP], PKG / "libgpuexp_hip.so",
                                 ["-lamdhip64", "-lhsa-runtime64"])),
        "kernels": str(link_hip([objs[s] for s in KERNELS_HIP], _ext("_gpuexp_kernels"), ["-lamdhip64"])),
    }
    if (CSRC / ROCPROF_CC[0]).exists():
        outputs["rocprof_plugin"] = str(link_plain([objs[ROCPROF_CC[0]]], PKG / "_gpuexp_rocprof.so",
                                                   ["-lrocprofiler-sdk", "-lhsa-runtime64", "-lpthread"]))
    if (CSRC / AQLPMC_CC[0]).exists():
        outputs["aqlpmc_plugin"] = str(link_plain([objs[AQLPMC_CC[0]], objs["gpuexp/pmc_rounds.cc"],
                                                   objs["gpuexp/pmc_agents.cc"]],
                                                  PKG / "_gpuexp_aqlpmc.so",
                                                  ["-lhsa-runtime64", "-lpthread"]))
        outputs["sentinel_hsaco"] = str(build_hsaco(SENTINEL_HSACO, PKG / "gpuexp_sentinel.hsaco", hdr, force))
        outputs["calib_hsaco"] = str(build_hsaco(CALIB_HSACO, PKG / "gpuexp_calib.hsaco", hdr, force))
    if (CSRC / TRACER_CC[0]).exists():
        outputs["rccl_tracer"] = str(link_plain([objs[TRACER_CC[0]]], PKG / "libgpuexp_rccl_tracer.so",
                                                ["-lrocprofiler-sdk", "-lpthread"]))
    if verbose:
        for k, v in outputs.items():
            print(f"[build_native] {k}: {v}")
    return outputs


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--sanitize", default=None, help="host sanitizer (address, undefined)")
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args()
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
    build(force=a.force, jobs=a.jobs, sanitize=a.sanitize)
    return 0


if __name__ == "__main__":
    sys.exit(main())
