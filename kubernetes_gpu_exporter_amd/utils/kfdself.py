"""Find this process's HOST PID as KFD reports it, from inside a PID namespace.

KFD's /sys/class/kfd/kfd/proc/<pid> directories are named by host PID.  In Kubernetes the
exporter runs with hostPID: true, so host PIDs are its PIDs.  A workload process inside
its own PID namespace (the gpurun box, or a test harness) cannot see its host PID in
/proc (NSpid shows one level) and the KFD `pasid` attribute reads 0 on this kernel
(measured, profiles/probe_pasid.txt).  This helper identifies the caller's KFD directory
by a VRAM fingerprint: allocate a buffer of a distinctive size and look for the directory
whose vram_<gpu_id> grew by exactly that amount.
"""
from __future__ import annotations

import glob
import os
import time


def _snapshot(gpu_id: int) -> dict:
    out = {}
    for path in glob.glob(f"/sys/class/kfd/kfd/proc/*/vram_{gpu_id}"):
        try:
            with open(path) as fh:
                out[int(path.split("/")[-2])] = int(fh.read().strip())
        except (OSError, ValueError):
            continue
    return out


def kfd_gpu_id_for_torch_device(index: int) -> int | None:
    """KFD gpu_id of torch device `index`, matched by PCI bus through amdsmi-free sysfs."""
    import torch
    props = torch.cuda.get_device_properties(index)
    bus = getattr(props, "pci_bus_id", None)
    dom = getattr(props, "pci_domain_id", 0)
    dev = getattr(props, "pci_device_id", 0)
    for node in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        try:
            gid = int(open(node + "/gpu_id").read().strip() or 0)
            if not gid:
                continue
            kv = dict(line.split() for line in open(node + "/properties") if len(line.split()) == 2)
            loc = int(kv.get("location_id", 0))
            if bus is None or ((loc >> 8) & 0xFF, (loc >> 3) & 0x1F, int(kv.get("domain", 0))) == (bus, dev, dom):
                return gid
        except (OSError, ValueError):
            continue
    return None


def find_own_kfd_pid(device_index: int = 0, salt: int = 0, tries: int = 3) -> int | None:
    """Returns the host PID KFD uses for this process (None if not identifiable)."""
    import torch
    if os.path.isdir(f"/sys/class/kfd/kfd/proc/{os.getpid()}"):
        return os.getpid()  # same PID namespace as the host
    gid = kfd_gpu_id_for_torch_device(device_index)
    if gid is None:
        return None
    mib = 1 << 20
    for attempt in range(tries):
        size = (513 + 7 * (salt % 97) + 3 * attempt) * 2 * mib  # 2 MiB-granular, rank-distinct
        torch.cuda.synchronize(device_index)
        before = _snapshot(gid)
        buf = torch.empty(size, dtype=torch.uint8, device=f"cuda:{device_index}")
        buf.fill_(1)
        torch.cuda.synchronize(device_index)
        time.sleep(0.05)
        after = _snapshot(gid)
        del buf
        torch.cuda.empty_cache()
        cands = [pid for pid, v in after.items() if v - before.get(pid, 0) == size]
        if len(cands) == 1:
            return cands[0]
    return None


def hip_order_bdfs(root: str = "") -> list:
    """PCI BDFs of the GPUs in HIP device order, WITHOUT initialising the GPU (a process
    that will spawn children must not touch HIP first).  ROCr enumerates GPU agents in
    KFD topology node order and HIP numbers them in that order; *_VISIBLE_DEVICES lists
    of integers are applied the way ROCr/HIP apply them."""
    nodes = []
    base = root + "/sys/class/kfd/kfd/topology/nodes"
    for name in os.listdir(base) if os.path.isdir(base) else []:
        if not name.isdigit():
            continue
        try:
            kv = dict(line.split() for line in open(f"{base}/{name}/properties") if len(line.split()) == 2)
        except OSError:
            continue
        if int(kv.get("simd_count", 0)) <= 0:
            continue  # CPU node
        minor = kv.get("drm_render_minor")
        if not root and minor is not None and not os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            continue  # ROCr skips GPUs whose render node this process cannot open
        loc, dom = int(kv.get("location_id", 0)), int(kv.get("domain", 0))
        nodes.append((int(name), f"{dom:04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 7:x}",
                      f"GPU-{int(kv.get('unique_id', 0)):016x}"))
    visible = [(b, u) for _, b, u in sorted(nodes)]
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var, "").strip()
        if not val:
            continue
        picked = []
        for x in (x.strip() for x in val.split(",")):
            if x.isdigit():
                if int(x) < len(visible):
                    picked.append(visible[int(x)])
            elif x.lower().startswith("gpu-"):  # ROCr UUIDs: "GPU-" + 16 hex digits of unique_id
                picked += [v for v in visible if v[1].lower() == x.lower()]
        visible = picked
    return [b for b, _ in visible]
