#!/usr/bin/env python3
"""GPU-box probe: resident memory of bare ROCm runtime initialisation (no exporter), to
find what inflates the exporter's RSS once its HIP sentinel / HSA counter plugins start.
Each case runs in a fresh child: hsa_init only, hipInit + a context on device 0, each with
selected env knobs; reports VmRSS and the largest individual mappings.
Usage: python tools/probe_runtime_rss.py"""
import json
import os
import subprocess
import sys

CHILD = r'''
import ctypes, json, os, sys
mode = sys.argv[1]
def rss():
    return int([l for l in open("/proc/self/status") if l.startswith("VmRSS:")][0].split()[1])
r0 = rss()
if mode == "hsa":
    h = ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so.1")
    assert h.hsa_init() == 0
else:
    h = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    assert h.hipInit(0) == 0
    assert h.hipSetDevice(0) == 0
    p = ctypes.c_void_p()
    assert h.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)) == 0
    h.hipDeviceSynchronize()
r1 = rss()
maps, cur = [], None
for line in open("/proc/self/smaps"):
    parts = line.split()
    if len(parts) >= 5 and "-" in parts[0] and ":" not in parts[0]:
        a, b = (int(x, 16) for x in parts[0].split("-"))
        cur = {"map": " ".join(parts[5:]) or "[anon]", "size_kb": (b - a) >> 10, "rss_kb": 0}
        maps.append(cur)
    elif parts and parts[0] == "Rss:" and cur is not None:
        cur["rss_kb"] = int(parts[1])
maps.sort(key=lambda m: -m["rss_kb"])
print("RESULT " + json.dumps({"mode": mode, "env": {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "HIP_", "GPU_", "AMD_", "ROC"))},
                              "rss_before_kb": r0, "rss_after_kb": r1, "top": maps[:6]}), flush=True)
'''


def main() -> int:
    cases = [("hsa", {}), ("hip", {}), ("hip", {"HIP_VISIBLE_DEVICES": "0"}),
             ("hip", {"HSA_KERNARG_POOL_SIZE": "1048576"}), ("hip", {"GPU_MAX_HW_QUEUES": "1"}),
             ("hsa", {"HSA_ENABLE_SDMA": "0"})]
    for mode, env in cases:
        r = subprocess.run([sys.executable, "-c", CHILD, mode], env=dict(os.environ, **env), capture_output=True,
                           text=True, timeout=120)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        print(line[-1] if line else f"FAILED {mode} {env}: {r.stderr[-400:]}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
