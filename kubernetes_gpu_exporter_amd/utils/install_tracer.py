"""Puts the RCCL tracer tool library on the node, where workload pods load it.

The DaemonSet runs this as an init container (deploy/kubernetes/daemonset.yaml,
deploy/helm/gpuexp/templates/daemonset.yaml) with the host directory the workload examples
mount read-only (/opt/gpuexp/lib); a workload then sets
ROCP_TOOL_LIBRARIES=/opt/gpuexp/libgpuexp_rccl_tracer.so and its collectives show up as
amd_rccl_collective_{calls,bytes}_total{namespace,pod,op}.  This is the delivery half of the
per-pod RCCL path; the reference discovered per-pod processes by `kubectl exec` instead
(/root/reference/main.go:91-110) and saw no collective traffic at all.

The copy goes to a temporary name in the target directory and is renamed over the old file:
a workload starting meanwhile maps either the old library or the new one, never a
half-written one, and a process that already mapped the old file keeps its inode.  An
identical file is left alone (no new inode for nothing).

    python -m kubernetes_gpu_exporter_amd.utils.install_tracer /host/opt/gpuexp/lib
"""
from __future__ import annotations

import filecmp
import os
import sys
import tempfile

TRACER = "libgpuexp_rccl_tracer.so"
ELF_MAGIC = b"\x7fELF"


def packaged_tracer() -> str:
    """The tracer built into this package (build_native.py puts it next to the modules)."""
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), TRACER)


def install(dest_dir: str, src: str | None = None) -> tuple[str, bool]:
    """Copies the tracer into dest_dir atomically; returns (path, changed)."""
    src = src or packaged_tracer()
    with open(src, "rb") as fh:
        if fh.read(4) != ELF_MAGIC:
            raise ValueError(f"{src} is not an ELF shared object")
    os.makedirs(dest_dir, exist_ok=True)
    dst = os.path.join(dest_dir, TRACER)
    if os.path.exists(dst) and filecmp.cmp(src, dst, shallow=False):
        return dst, False
    fd, tmp = tempfile.mkstemp(prefix=f".{TRACER}.", dir=dest_dir)
    try:
        with os.fdopen(fd, "wb") as out, open(src, "rb") as inp:
            while True:
                chunk = inp.read(1 << 20)
                if not chunk:
                    break
                out.write(chunk)
            out.flush()
            os.fsync(out.fileno())
        os.chmod(tmp, 0o755)
        os.replace(tmp, dst)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
    return dst, True


def main(argv: list | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        print("usage: python -m kubernetes_gpu_exporter_amd.utils.install_tracer DEST_DIR", file=sys.stderr)
        return 2
    path, changed = install(argv[0])
    print(f"rccl tracer {'installed' if changed else 'already current'}: {path}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
