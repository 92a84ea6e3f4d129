"""The RCCL tracer's node install (utils/install_tracer.py, the DaemonSet's init container)
and the library's load-time contract with a workload's ROCm (NEEDED libraries, symbol
versions, the rocprofiler-sdk entry points it calls)."""
import os
import shutil
import subprocess

import pytest

from kubernetes_gpu_exporter_amd.utils import install_tracer as it

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "kubernetes_gpu_exporter_amd", it.TRACER)


def test_install_is_atomic_and_idempotent(tmp_path):
    src = tmp_path / "src.so"
    src.write_bytes(b"\x7fELF" + b"x" * 5000)
    dest = tmp_path / "host" / "opt" / "gpuexp" / "lib"
    path, changed = it.install(str(dest), str(src))
    assert changed and open(path, "rb").read() == src.read_bytes()
    assert oct(os.stat(path).st_mode & 0o777) == "0o755"
    ino = os.stat(path).st_ino
    path2, changed2 = it.install(str(dest), str(src))  # identical: left alone (same inode)
    assert not changed2 and os.stat(path2).st_ino == ino
    src.write_bytes(b"\x7fELF" + b"y" * 5000)
    held = open(path, "rb")  # a workload that mapped the old file keeps reading the old inode
    _, changed3 = it.install(str(dest), str(src))
    assert changed3 and os.stat(path).st_ino != ino
    assert held.read()[4:5] == b"x"
    held.close()
    assert sorted(os.listdir(dest)) == [it.TRACER]  # no temporary left behind


def test_install_refuses_a_non_elf_file(tmp_path):
    src = tmp_path / "bad.so"
    src.write_text("not a library")
    with pytest.raises(ValueError):
        it.install(str(tmp_path / "d"), str(src))
    assert not (tmp_path / "d" / it.TRACER).exists()


def test_install_cli(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("tracer not built")
    r = subprocess.run(["python3", "-m", "kubernetes_gpu_exporter_amd.utils.install_tracer", str(tmp_path)],
                       cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "installed" in r.stdout and (tmp_path / it.TRACER).exists()


def _readelf(*args):
    exe = shutil.which("readelf")
    if not exe or not os.path.exists(LIB):
        pytest.skip("readelf or the tracer missing")
    return subprocess.run([exe, *args, LIB], capture_output=True, text=True, check=True).stdout


def test_tracer_load_contract():
    """What a workload's image must provide for the tracer to load: its NEEDED libraries
    (rocprofiler-sdk.so.1 + the C/C++ runtime), glibc <= 2.34 and libstdc++ <= GLIBCXX_3.4.29
    symbol versions (Ubuntu 22.04 / RHEL 9 class images), and only three rocprofiler-sdk
    entry points, present since the callback tracing API.  The RCCL domain id it passes is
    the one of rocprofiler-sdk 1.1 (ROCm 7.2), so rocprofiler_configure declines older
    runtimes (the workload then runs untraced instead of tracing the wrong domain)."""
    import re
    needed = set(re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", _readelf("-d")))
    assert needed == {"librocprofiler-sdk.so.1", "libstdc++.so.6", "libgcc_s.so.1", "libc.so.6",
                      "ld-linux-x86-64.so.2"}, needed
    syms = _readelf("--dyn-syms", "-W")
    vers = lambda tag: [tuple(int(x) for x in v.split(".")) for v in re.findall(tag + r"_([0-9.]+)", syms)]  # noqa: E731
    assert max(vers("GLIBC")) <= (2, 34), max(vers("GLIBC"))
    assert max(vers("GLIBCXX")) <= (3, 4, 29), max(vers("GLIBCXX"))
    undef = {m for m in re.findall(r"\bUND\s+(rocprofiler_[a-z_]+)", syms)}
    assert undef == {"rocprofiler_configure_callback_tracing_service", "rocprofiler_create_context",
                     "rocprofiler_start_context"}, undef
    defined = re.findall(r"\bGLOBAL\s+DEFAULT\s+\d+\s+(\w+)", syms)
    assert "rocprofiler_configure" in defined


def test_tracer_declines_an_older_rocprofiler_sdk():
    """rocprofiler_configure(version, ...) returns a configuration for rocprofiler-sdk 1.x at or
    above the version the tracer was built against, and NULL (the tool stays unloaded) below it."""
    import ctypes
    if not os.path.exists(LIB):
        pytest.skip("tracer not built")
    try:
        lib = ctypes.CDLL(LIB)
    except OSError as ex:
        pytest.skip(f"cannot load the tracer here: {ex}")

    class ClientId(ctypes.Structure):
        _fields_ = [("name", ctypes.c_char_p), ("handle", ctypes.c_uint32)]

    f = lib.rocprofiler_configure
    f.restype = ctypes.c_void_p
    f.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ClientId)]
    built = lib.gpuexp_rccl_tracer_built_sdk_version
    built.restype = ctypes.c_uint32
    v = built()
    assert v >= 10100, v  # built against rocprofiler-sdk >= 1.1.0
    cid = ClientId()
    assert f(v, b"test", 0, ctypes.byref(cid))  # the version it was built against
    assert f(v + 1, b"test", 0, ctypes.byref(cid))  # a newer patch / minor of 1.x
    assert not f(v - 100, b"test", 0, ctypes.byref(cid))  # an older minor
    assert not f(600, b"test", 0, ctypes.byref(cid))  # 0.6.0 (ROCm 6.x)
    assert not f(20000, b"test", 0, ctypes.byref(cid))  # a future major
