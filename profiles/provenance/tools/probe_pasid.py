"""GPU-box probe: (1) can a process in a non-host PID namespace be matched to its KFD host
PID through the VM pasid (fdinfo of its render node vs /sys/class/kfd/kfd/proc/*/pasid)?
(2) what does each sysfs read on the per-tick path cost?"""
import glob
import os
import time

import torch

x = torch.ones(1 << 28, device="cuda")  # hold a KFD context + 1 GiB
torch.cuda.synchronize()
print("self pid", os.getpid(), "NSpid", open("/proc/self/status").read().split("NSpid:")[1].split("\n")[0].split())
print("pidns", os.stat("/proc/self/ns/pid").st_ino, "(init ns = 4026531836)")
for fd in sorted(os.listdir("/proc/self/fd"), key=int):
    try:
        target = os.readlink(f"/proc/self/fd/{fd}")
    except OSError:
        continue
    if "/dev/dri" in target or "/dev/kfd" in target:
        info = open(f"/proc/self/fdinfo/{fd}").read()
        print(f"fd {fd} -> {target}\n  " + "\n  ".join(info.strip().splitlines()))
for d in sorted(glob.glob("/sys/class/kfd/kfd/proc/*")):
    try:
        pas = open(d + "/pasid").read().strip()
    except OSError as e:
        pas = repr(e)
    vr = {os.path.basename(v): open(v).read().strip() for v in glob.glob(d + "/vram_*")}
    print("kfd", os.path.basename(d), "pasid", pas, vr)


def cost(path, n=200):
    fd = os.open(path, os.O_RDONLY)
    os.pread(fd, 8192, 0)
    t0 = time.perf_counter()
    for _ in range(n):
        os.pread(fd, 8192, 0)
    dt = (time.perf_counter() - t0) / n * 1e6
    os.close(fd)
    return dt


dev = glob.glob("/sys/class/drm/renderD*/device/gpu_metrics")[0].rsplit("/", 1)[0]
for f in ["gpu_metrics", "mem_info_vram_used", "gpu_busy_percent", "mem_busy_percent"]:
    print(f"read cost {f}: {cost(dev + '/' + f):.1f} us")
for h in glob.glob(dev + "/hwmon/hwmon*/power1_input") + glob.glob(dev + "/hwmon/hwmon*/temp2_input"):
    print(f"read cost {h.rsplit('/', 1)[1]}: {cost(h):.1f} us")
kp = glob.glob("/sys/class/kfd/kfd/proc/*/vram_*")
if kp:
    print(f"read cost kfd vram: {cost(kp[0]):.1f} us")
cu = glob.glob("/sys/class/kfd/kfd/proc/*/stats_*/cu_occupancy")
if cu:
    print(f"read cost kfd cu_occupancy: {cost(cu[0], 50):.1f} us")
