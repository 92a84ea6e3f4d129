#!/usr/bin/env python3
"""Runs a few bf16 GEMM dispatches of one kernel variant, for `rocprofv3 --pmc` runs:
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ... -d out -- python3 tools/gemm_pmc.py 8192 0
variant: 0 auto (256x256, 8-row groups), 1 = 128x128, 2-4 = 256x256 tile orders."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    from kubernetes_gpu_exporter_amd.ops.gemm import kernels
    r = kernels().gemm_burn(0, n, n, n, 0.2, 4, variant)
    print(f"gemm {n}^3 variant {variant}: {r}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
