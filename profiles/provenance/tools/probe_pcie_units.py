#!/usr/bin/env python3
"""What unit is gpu_metrics pcie_bandwidth_inst in?  A child streams pinned host memory to
the GPU (H2D), then GPU to host (D2H), at measured payload rates; meanwhile this process
reads the raw gpu_metrics value (our decoder) and amdsmi_get_pcie_info's pcie_bandwidth
(documented Mb/s).  Prints one line per phase."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = """
import json, sys, time, torch
host = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
dev.copy_(host); torch.cuda.synchronize()
for phase in ("h2d", "d2h"):
    print("start " + phase, flush=True)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        if phase == "h2d": dev.copy_(host, non_blocking=True)
        else: host.copy_(dev, non_blocking=True)
        torch.cuda.synchronize(); n += 1
    print(json.dumps({"phase": phase, "Bps": n * (1 << 30) / (time.perf_counter() - t0)}), flush=True)
    time.sleep(0.5)
"""


def main():
    import amdsmi
    from kubernetes_gpu_exporter_amd._native import load
    n = load()
    info = n.read_backend("amdsmi")[0]
    path = f"/sys/class/drm/renderD{info['render_minor']}/device/gpu_metrics"
    os.environ["AMDSMI_GPU_METRICS_CACHE_MS"] = "0"
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    child = subprocess.Popen([sys.executable, "-c", CHILD], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    for line in child.stdout:
        line = line.strip()
        if line.startswith("start "):
            phase = line[6:]
            time.sleep(0.5)
            raw, smi, acc = [], [], []
            for _ in range(15):
                with open(path, "rb") as fh:
                    r = n.decode_gpu_metrics_raw(fh.read())
                raw.append(r["pcie_bandwidth_inst"])
                acc.append(r["pcie_bandwidth_acc"])
                try:
                    smi.append(amdsmi.amdsmi_get_pcie_info(h)["pcie_metric"]["pcie_bandwidth"])
                except Exception as ex:  # noqa: BLE001
                    smi.append(str(ex))
                time.sleep(0.1)
            print("SAMPLES", phase, json.dumps({"raw_inst": raw[len(raw) // 2], "amdsmi_pcie_bandwidth": smi[len(smi) // 2],
                                                "acc_first_last": [acc[0], acc[-1]]}), flush=True)
        elif line.startswith("{"):
            print("MEASURED", line, flush=True)
    child.wait()
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
