"""Fake host roots: a temp tree shaped like an MI355X node's /sys + /proc, for the
fake-host integration tier.  Layout mirrors what the probe found on the
GPU box (profiles/probe_host.txt): KFD topology nodes with gpu_id/properties, drm
renderD<minor>/device with gpu_metrics + mem_info_* + hwmon, KFD per-process
vram_<gpu_id>/sdma_<gpu_id>/stats_<gpu_id>/cu_occupancy, /proc/<pid>/{cgroup,comm,stat}.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from pathlib import Path

GPU_METRICS_V1_8_SIZE = 3872


def encode_gpu_metrics_v1_8(*, hotspot=46, mem=34, vrsoc=41, power=244, gfx=0, umc=0, max_bw=8192,
                            energy=18067985097658, sysclk=1051434741968776, accum=1051349996,
                            ppt_res=2146364, pcie_width=16, pcie_speed=320, xgmi_width=16, xgmi_speed=38,
                            pcie_bw_acc=912039705430, pcie_bw_inst=18, xgmi_rd=None, xgmi_wr=None,
                            xgmi_status=None, fw_ts=105165583750064, gfxclk=(111,) * 8, socclk=38,
                            uclk=2000, gfx_busy_acc=(0,) * 8, num_partition=1, xcp_busy_acc=None) -> bytes:
    """Packs a gpu_metrics format-1.8 blob with the field offsets the C++ decoder uses.
    xcp_busy_acc: {partition: 8 per-XCD busy accumulators} for partitioned sockets
    (xcp_stats[k], 440 bytes each); gfx_busy_acc is partition 0's."""
    xgmi_rd = list(xgmi_rd or [0] * 8)
    xgmi_wr = list(xgmi_wr or [0] * 8)
    xgmi_status = list(xgmi_status or [0xFFFF] + [1] * 7)
    b = bytearray(GPU_METRICS_V1_8_SIZE)
    struct.pack_into("<HBB", b, 0, GPU_METRICS_V1_8_SIZE, 1, 8)
    struct.pack_into("<6H", b, 4, hotspot, mem, vrsoc, power, gfx, umc)
    struct.pack_into("<3Q", b, 16, max_bw, energy, sysclk)
    struct.pack_into("<7I", b, 40, accum, 0, ppt_res, 0, 0, 0, 0)
    struct.pack_into("<4H", b, 68, pcie_width, pcie_speed, xgmi_width, xgmi_speed)
    struct.pack_into("<2I", b, 76, 0, 0)
    struct.pack_into("<5Q", b, 88, pcie_bw_acc, pcie_bw_inst, 0, 0, 0)
    struct.pack_into("<2I", b, 128, 0, 0)
    struct.pack_into("<8Q", b, 136, *xgmi_rd)
    struct.pack_into("<8Q", b, 200, *xgmi_wr)
    struct.pack_into("<8H", b, 264, *xgmi_status)
    struct.pack_into("<Q", b, 288, fw_ts)
    struct.pack_into("<8H", b, 296, *gfxclk)
    struct.pack_into("<4H", b, 312, socclk, 0xFFFF, 0xFFFF, 0xFFFF)
    struct.pack_into("<H", b, 336, uclk)
    struct.pack_into("<H", b, 338, num_partition)
    # xcp_stats[k].gfx_busy_acc at 344 + 440 * k + 120
    struct.pack_into("<8Q", b, 344 + 120, *gfx_busy_acc)
    for k, acc in (xcp_busy_acc or {}).items():
        struct.pack_into("<8Q", b, 344 + 440 * k + 120, *acc)
    return bytes(b)


@dataclass
class FakeGpu:
    gpu_id: int
    location_id: int            # (bus << 8) | (dev << 3) | fn
    render_minor: int
    unique_id: int = 0xE296A367FEF9A1BE
    device_id: int = 0x75A3
    vram_total: int = 309220868096
    vram_used: int = 297766912
    metrics: dict = field(default_factory=dict)
    num_xcc: int = 8                 # 1 per partition in CPX mode
    compute_partition: str = "SPX"   # SPX | DPX | QPX | CPX
    memory_partition: str = "NPS1"
    # sysfs device behind the render node: "" = a plain directory (older fixtures); a BDF
    # = a PCI function under sys/devices (also linked from sys/bus/pci/devices); 
    # "amdgpu_xcp.<n>" = the platform device of a partition >= 1 of a partitioned socket
    dev_node: str = ""
    # partitions >= 1: keep gpu_metrics / mem_info_* / hwmon on the socket's PCI function
    # only (the XCP platform device carries none of them)
    files_on_pci: bool = False


class FakeHost:
    def __init__(self, root: str | os.PathLike):
        self.root = Path(root)
        self.gpus: list[FakeGpu] = []

    def _bdf(self, gpu: FakeGpu) -> str:
        return f"0000:{(gpu.location_id >> 8) & 0xFF:02x}:{(gpu.location_id >> 3) & 0x1F:02x}.{gpu.location_id & 7:x}"

    def dev_dir(self, gpu: FakeGpu) -> str:
        """Where the device's sysfs files go (relative to the root)."""
        if gpu.files_on_pci:
            return f"sys/bus/pci/devices/{self._bdf(gpu)}"
        return f"sys/class/drm/renderD{gpu.render_minor}/device"

    def _link_device(self, gpu: FakeGpu) -> None:
        if not gpu.dev_node:
            return
        xcp = gpu.dev_node.startswith("amdgpu_xcp")
        real = self.root / ("sys/devices/platform" if xcp else "sys/devices/pci0000:00") / gpu.dev_node
        real.mkdir(parents=True, exist_ok=True)
        link = self.root / f"sys/class/drm/renderD{gpu.render_minor}/device"
        link.parent.mkdir(parents=True, exist_ok=True)
        if not link.is_symlink():
            link.symlink_to(real)
        if not xcp:
            pci = self.root / "sys/bus/pci/devices" / gpu.dev_node
            pci.parent.mkdir(parents=True, exist_ok=True)
            if not pci.is_symlink():
                pci.symlink_to(real)

    def _w(self, rel: str, data, mode: str = "w") -> Path:
        p = self.root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        with open(p, mode) as fh:
            fh.write(data)
        return p

    # ---- devices ----
    def add_gpu(self, node: int, gpu: FakeGpu) -> FakeGpu:
        nd = f"sys/class/kfd/kfd/topology/nodes/{node}"
        self._w(f"{nd}/gpu_id", f"{gpu.gpu_id}\n")
        self._w(f"{nd}/name", "ip discovery\n")
        props = {"simd_count": 1024, "simd_per_cu": 4, "array_count": 32, "location_id": gpu.location_id,
                 "domain": 0, "drm_render_minor": gpu.render_minor, "unique_id": gpu.unique_id,
                 "device_id": gpu.device_id, "num_xcc": gpu.num_xcc, "gfx_target_version": 90500,
                 "max_engine_clk_fcompute": 2400}
        self._w(f"{nd}/properties", "".join(f"{k} {v}\n" for k, v in props.items()))
        self._link_device(gpu)
        dev = self.dev_dir(gpu)
        self._w(f"{dev}/mem_info_vram_total", f"{gpu.vram_total}\n")
        self._w(f"{dev}/mem_info_vram_used", f"{gpu.vram_used}\n")
        self._w(f"{dev}/gpu_busy_percent", "0\n")
        self._w(f"{dev}/mem_busy_percent", "0\n")
        self._w(f"{dev}/current_compute_partition", gpu.compute_partition + "\n")
        self._w(f"{dev}/current_memory_partition", gpu.memory_partition + "\n")
        self._w(f"{dev}/hwmon/hwmon0/power1_input", "244000000\n")
        self._w(f"{dev}/hwmon/hwmon0/power1_cap", "1400000000\n")
        self._w(f"{dev}/hwmon/hwmon0/temp2_label", "junction\n")
        self._w(f"{dev}/hwmon/hwmon0/temp2_input", "46000\n")
        self._w(f"{dev}/hwmon/hwmon0/temp3_label", "mem\n")
        self._w(f"{dev}/hwmon/hwmon0/temp3_input", "34000\n")
        self.set_metrics(gpu, **gpu.metrics)
        self.gpus.append(gpu)
        return gpu

    def add_cpu_node(self, node: int) -> None:
        nd = f"sys/class/kfd/kfd/topology/nodes/{node}"
        self._w(f"{nd}/gpu_id", "0\n")
        self._w(f"{nd}/properties", "simd_count 0\nlocation_id 0\n")

    def set_metrics(self, gpu: FakeGpu, **kw) -> None:
        gpu.metrics = kw
        self._w(f"{self.dev_dir(gpu)}/gpu_metrics", encode_gpu_metrics_v1_8(**kw), "wb")

    def set_ras(self, gpu: FakeGpu, blocks: dict | None = None, aer: tuple = (0, 0, 0)) -> None:
        """amdgpu ras/<block>_err_count ("ue: N\nce: N") and PCI aer_dev_* totals."""
        dev = self.dev_dir(gpu)
        for block, (ue, ce) in (blocks or {"umc": (0, 0), "gfx": (0, 0)}).items():
            self._w(f"{dev}/ras/{block}_err_count", f"ue: {ue}\nce: {ce}\n")
        self._w(f"{dev}/ras/features", "feature mask: 0x3fff\n")
        names = ("correctable", "nonfatal", "fatal")
        keys = ("TOTAL_ERR_COR", "TOTAL_ERR_NONFATAL", "TOTAL_ERR_FATAL")
        for n, k, v in zip(names, keys, aer):
            self._w(f"{dev}/aer_dev_{n}", f"RxErr 0\nBadTLP 0\n{k} {v}\n")

    def set_xgmi_ports(self) -> dict:
        """amdgpu's xgmi_port_num for every socket (one per distinct BDF) of the hive, in the
        kernel's "<node>:<port> ->  <peer node>:<peer port>" form: node ids 1..n in GPU order,
        socket i's port p (1..n-1) wired to socket (i + p) % n.  Returns {bdf: {port: peer bdf}}."""
        bdfs = list(dict.fromkeys(self._bdf(g) for g in self.gpus))
        n = len(bdfs)
        wiring = {}
        for i, b in enumerate(bdfs):
            lines, ports = [], {}
            for p in range(1, n):
                j = (i + p) % n
                lines.append(f"{i + 1:02x}:{p:02x} ->  {j + 1:02x}:{n - p:02x}\n")
                ports[p] = bdfs[j]
            self._w(f"sys/bus/pci/devices/{b}/xgmi_port_num", "".join(lines))
            wiring[b] = ports
        return wiring

    def set_board(self, gpu: FakeGpu, serial: str = "PV0A1B2C3D", firmware: dict | None = None) -> None:
        """Board identity (vbios_version, product_name/_number, serial_number) and
        fw_version/<component>_fw_version on the PCI function."""
        b = f"sys/bus/pci/devices/{self._bdf(gpu)}"
        self._w(f"{b}/vbios_version", "113-M3550100-100\n")
        self._w(f"{b}/product_name", "AMD Instinct MI355X\n")
        self._w(f"{b}/product_number", "102-M3550-00\n")
        self._w(f"{b}/serial_number", f"{serial}\n")
        for comp, ver in (firmware or {"mec": "0x0000009f", "smc": "0x00554500", "vcn": "0x00000000"}).items():
            self._w(f"{b}/fw_version/{comp}_fw_version", f"{ver}\n")

    def set_bad_pages(self, gpu: FakeGpu, states: str) -> None:
        """ras/gpu_vram_bad_pages, one retired-page line per character of `states`
        (R reserved, P pending, F unreservable), in amdgpu's "0x<page> : 0x<size> : S" form."""
        lines = "".join(f"0x{0x1000 + k:08x} : 0x00001000 : {st}\n" for k, st in enumerate(states))
        self._w(f"{self.dev_dir(gpu)}/ras/gpu_vram_bad_pages", lines)

    def set_gtt(self, gpu: FakeGpu, used: int, total: int) -> None:
        self._w(f"{self.dev_dir(gpu)}/mem_info_gtt_used", f"{used}\n")
        self._w(f"{self.dev_dir(gpu)}/mem_info_gtt_total", f"{total}\n")

    def set_vram_used(self, gpu: FakeGpu, used: int) -> None:
        self._w(f"{self.dev_dir(gpu)}/mem_info_vram_used", f"{used}\n")

    def remove_gpu_metrics(self, gpu: FakeGpu) -> None:
        (self.root / self.dev_dir(gpu) / "gpu_metrics").unlink()

    # ---- processes ----
    def add_process(self, pid: int, cgroup: str, comm: str = "python3", gpus: dict | None = None,
                    starttime: int = 1000, comm_readable: bool = True) -> None:
        """gpus: {gpu_id: (vram_bytes, cu_occupancy)}.  comm_readable=False makes reads of the
        process's comm fail the way they do once it has exited (ESRCH on an open fd): the fake's
        comm is a directory, which opens but fails every read (an unlinked file stays readable)."""
        self._w(f"proc/{pid}/cgroup", f"0::{cgroup}\n")
        if comm_readable:
            self._w(f"proc/{pid}/comm", comm + "\n")
        else:
            (self.root / f"proc/{pid}/comm").mkdir(parents=True, exist_ok=True)
        fields = ["S"] + ["0"] * 18 + [str(starttime)] + ["0"] * 10
        self._w(f"proc/{pid}/stat", f"{pid} ({comm}) " + " ".join(fields) + "\n")
        for gid, (vram, cu) in (gpus or {}).items():
            self.set_process_gpu(pid, gid, vram, cu)

    def set_process_gpu(self, pid: int, gpu_id: int, vram: int, cu: int = 0, sdma_us: int = 0,
                        evicted_ms: int = 0) -> None:
        pd = f"sys/class/kfd/kfd/proc/{pid}"
        self._w(f"{pd}/vram_{gpu_id}", f"{vram}\n")
        self._w(f"{pd}/sdma_{gpu_id}", f"{sdma_us}\n")
        self._w(f"{pd}/stats_{gpu_id}/cu_occupancy", f"{cu}\n")
        self._w(f"{pd}/stats_{gpu_id}/evicted_ms", f"{evicted_ms}\n")
        self._w(f"{pd}/pasid", "32769\n")

    def remove_process(self, pid: int) -> None:
        import shutil
        # As on the real filesystems, files a reader still holds open stop reading once the
        # process is gone (sysfs: the KFD kobject is removed, -ENODEV; procfs: -ESRCH), where
        # an unlinked tmpfs file would keep its old contents: empty them first.
        for d in (self.root / f"sys/class/kfd/kfd/proc/{pid}", self.root / f"proc/{pid}"):
            for f in d.rglob("*") if d.exists() else ():
                if f.is_file():
                    try:
                        f.write_bytes(b"")
                    except OSError:
                        pass
        shutil.rmtree(self.root / f"sys/class/kfd/kfd/proc/{pid}", ignore_errors=True)
        shutil.rmtree(self.root / f"proc/{pid}", ignore_errors=True)

    def add_pod_logdir(self, namespace: str, pod: str, uid: str, containers=("main",)) -> None:
        for c in containers:
            d = self.root / f"var/log/pods/{namespace}_{pod}_{uid}/{c}"
            d.mkdir(parents=True, exist_ok=True)


def kubepods_cgroup(uid: str, container_id: str, qos: str = "burstable", driver: str = "systemd",
                    runtime: str = "containerd") -> str:
    """Builds a realistic cgroup-v2 path for a container of pod `uid`."""
    prefix = {"containerd": "cri-containerd-", "crio": "crio-", "docker": "docker-"}[runtime]
    if driver == "systemd":
        u = uid.replace("-", "_")
        if qos == "guaranteed":
            return f"/kubepods.slice/kubepods-pod{u}.slice/{prefix}{container_id}.scope"
        return (f"/kubepods.slice/kubepods-{qos}.slice/kubepods-{qos}-pod{u}.slice/"
                f"{prefix}{container_id}.scope")
    if qos == "guaranteed":
        return f"/kubepods/pod{uid}/{container_id}"
    return f"/kubepods/{qos}/pod{uid}/{container_id}"


def mi355x_cpx_socket(root, bus: int = 0x72, partitions: int = 8, xcp_files: bool = True) -> FakeHost:
    """One MI355X socket in CPX mode: `partitions` logical GPUs (one XCD each), each with
    its own KFD node, gpu_id and render node but the socket's PCI BDF and gpu_metrics.
    As amdgpu lays it out, partition 0's render node sits on the PCI function and the
    others' on platform devices amdgpu_xcp.<k>; xcp_files=False leaves those without any
    socket files (they are read from the PCI function then)."""
    h = FakeHost(root)
    h.add_cpu_node(0)
    bdf = f"0000:{bus:02x}:00.0"
    for k in range(partitions):
        h.add_gpu(1 + k, FakeGpu(gpu_id=41000 + 13 * k, location_id=bus << 8, render_minor=128 + k,
                                 num_xcc=8 // partitions, compute_partition="CPX" if partitions == 8 else
                                 {2: "DPX", 4: "QPX"}.get(partitions, "SPX"), memory_partition="NPS4",
                                 vram_total=309220868096 // 4, dev_node=bdf if k == 0 else f"amdgpu_xcp.{k}",
                                 files_on_pci=k > 0 and not xcp_files))
    return h


def mi355x_cpx_node(root, sockets: int = 8, partitions: int = 8) -> FakeHost:
    """An MI355X node with every socket in CPX (or DPX/QPX) mode: sockets x partitions logical
    GPUs (64 for 8 sockets in CPX), laid out as mi355x_cpx_socket lays out one socket, with
    node-wide KFD node ids, gpu_ids, render minors and amdgpu_xcp.<n> platform devices."""
    h = FakeHost(root)
    h.add_cpu_node(0)
    buses = [0x72, 0x5A, 0x23, 0xD9, 0xF1, 0xA4, 0x8B, 0x0A]
    mode = "CPX" if partitions == 8 else {2: "DPX", 4: "QPX"}.get(partitions, "SPX")
    for s in range(sockets):
        bus = buses[s % len(buses)] + (s // len(buses))
        bdf = f"0000:{bus:02x}:00.0"
        for k in range(partitions):
            n = s * partitions + k
            h.add_gpu(1 + n, FakeGpu(gpu_id=41000 + 13 * n, location_id=bus << 8, render_minor=128 + n,
                                     num_xcc=8 // partitions, compute_partition=mode, memory_partition="NPS4",
                                     vram_total=309220868096 // 4, unique_id=0xE296A367FEF9A1BE + s,
                                     dev_node=bdf if k == 0 else f"amdgpu_xcp.{n}"))
    return h


def mi355x_node(root, n_gpus: int = 8) -> FakeHost:
    """An 8-GPU MI355X node (gpu_ids/BDFs shaped like the probe's real values)."""
    h = FakeHost(root)
    h.add_cpu_node(0)
    h.add_cpu_node(1)
    buses = [0x72, 0x5A, 0x23, 0xD9, 0xF1, 0xA4, 0x8B, 0x0A]
    for i in range(n_gpus):
        h.add_gpu(2 + i, FakeGpu(gpu_id=28720 + 17 * i, location_id=buses[i] << 8, render_minor=128 + 8 * i,
                                 unique_id=0xE296A367FEF9A1BE + i))
    return h
