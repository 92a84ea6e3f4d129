"""Single-process workload for rocprofv3: the synthetic GEMM pod (bf16 MFMA kernel) running
while an in-process exporter engine samples at 10 Hz with the HIP sentinel enabled.
No child processes (safe under rocprofv3's preload).  Usage:
  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -- \
      python tools/profile_workload.py --seconds 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--sizes", default="8192,4096")
    ap.add_argument("--sentinel", type=int, default=1)
    a = ap.parse_args()
    import torch
    torch.zeros(1, device="cuda")
    from kubernetes_gpu_exporter_amd._native import load
    from kubernetes_gpu_exporter_amd.ops.gemm import kernels
    n = load()
    c = n.EngineConfig()
    c.backend = "amdsmi"
    c.interval_s = 0.1
    c.serve_http = False
    c.enable_sentinel = bool(a.sentinel)
    c.device_filter = [0]
    e = n.Engine(c)
    e.start()
    k = kernels()
    for s in a.sizes.split(","):
        s = int(s)
        r = k.gemm_burn(0, s, s, s, a.seconds, 4)
        print(f"gemm {s}^3: {r['tflops']:.1f} TFLOP/s over {r['iters']} iters", flush=True)
    e.stop()
    st = e.stats()
    print("exporter ticks", st["ticks"], "stage_ns", st["stage_ns"], flush=True)


if __name__ == "__main__":
    main()
