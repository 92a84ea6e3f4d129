#!/usr/bin/env python3
"""GPU-box probe: host memory that each GPU queue costs.  Every HSA/HIP hardware queue
gets a context save/restore (CWSR) area in GTT sized by KFD for the whole GPU; on MI355X
that is large, so the exporter's queue count drives its RSS.  Reports RSS after HIP init,
after the first kernel on a created stream, on a second (low-priority) stream and on the
null stream, and after one raw hsa_queue_create; plus KFD's cwsr/ctl_stack sizes.
Usage: python tools/probe_queue_rss.py"""
import json
import os
import subprocess
import sys

CHILD_HIP = r'''
import ctypes, json
def rss():
    return int([l for l in open("/proc/self/status") if l.startswith("VmRSS:")][0].split()[1])
h = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
out = {}
assert h.hipInit(0) == 0 and h.hipSetDevice(0) == 0
p = ctypes.c_void_p()
assert h.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)) == 0
out["init"] = rss()
s1 = ctypes.c_void_p()
assert h.hipStreamCreate(ctypes.byref(s1)) == 0
assert h.hipMemsetAsync(p, 0, ctypes.c_size_t(1 << 20), s1) == 0
h.hipStreamSynchronize(s1)
out["stream1_kernel"] = rss()
s2 = ctypes.c_void_p()
assert h.hipStreamCreateWithPriority(ctypes.byref(s2), 0, 1) == 0
assert h.hipMemsetAsync(p, 0, ctypes.c_size_t(1 << 20), s2) == 0
h.hipStreamSynchronize(s2)
out["stream2_lowprio_kernel"] = rss()
assert h.hipMemsetAsync(p, 0, ctypes.c_size_t(1 << 20), None) == 0
h.hipDeviceSynchronize()
out["null_stream_kernel"] = rss()
print("RESULT " + json.dumps(out), flush=True)
'''

CHILD_HSA = r'''
import ctypes, json
def rss():
    return int([l for l in open("/proc/self/status") if l.startswith("VmRSS:")][0].split()[1])
h = ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so.1")
assert h.hsa_init() == 0
out = {"init": rss()}
agents = []
CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)
def cb(agent, data):
    dev = ctypes.c_int(0)
    h.hsa_agent_get_info(ctypes.c_uint64(agent), 17, ctypes.byref(dev))  # HSA_AGENT_INFO_DEVICE
    if dev.value == 1:  # HSA_DEVICE_TYPE_GPU
        agents.append(agent)
    return 0
h.hsa_iterate_agents(CB(cb), None)
q = ctypes.c_void_p()
rc = h.hsa_queue_create(ctypes.c_uint64(agents[0]), ctypes.c_uint32(4096), ctypes.c_uint32(1), None, None,
                        ctypes.c_uint32(0xFFFFFFFF), ctypes.c_uint32(0xFFFFFFFF), ctypes.byref(q))
out["queue_rc"] = rc
out["one_queue"] = rss()
print("RESULT " + json.dumps(out), flush=True)
'''


def topo() -> list:
    base = "/sys/class/kfd/kfd/topology/nodes"
    out = []
    for n in sorted(os.listdir(base), key=lambda x: int(x) if x.isdigit() else 0):
        try:
            kv = dict(l.split() for l in open(f"{base}/{n}/properties") if len(l.split()) == 2)
        except OSError:
            continue
        if int(kv.get("simd_count", 0)) > 0:
            out.append({k: kv.get(k) for k in ("cwsr_size", "ctl_stack_size", "simd_count", "num_xcc",
                                                "max_waves_per_simd")})
    return out


def main() -> int:
    print("TOPOLOGY " + json.dumps(topo()), flush=True)
    for name, code in (("hip", CHILD_HIP), ("hsa", CHILD_HSA)):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        print(f"{name} " + (line[-1] if line else f"FAILED {r.stderr[-600:]}"), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
