#!/usr/bin/env python3
"""How often does KFD's per-process cu_occupancy read 0 for a process that keeps the GPU
busy?  Starts a torch-free GEMM burn (ops.gemm.gemm_burn) in a child process, then reads
/sys/class/kfd/kfd/proc/<child>/stats_<gpu_id>/cu_occupancy every `period_ms` for
`seconds`, next to the PMFW gfx activity.  Prints the value histogram and runs of zeros.
Usage: python tools/probe_cu_occupancy.py [seconds=3] [period_ms=5]
"""
import collections
import glob
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    period = float(sys.argv[2]) / 1000.0 if len(sys.argv) > 2 else 0.005
    before = set(glob.glob("/sys/class/kfd/kfd/proc/*"))
    child = subprocess.Popen([sys.executable, "-c",
                              "import sys; sys.path.insert(0, %r);"
                              "from kubernetes_gpu_exporter_amd.ops.gemm import gemm_burn;"
                              "print(gemm_burn(0, 8192, %f, 4), flush=True)" % (ROOT, secs + 20)],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        files = []
        t0 = time.time()
        while time.time() - t0 < 60 and not files:
            # KFD names the directory by HOST pid (the box may run in a pid namespace): the
            # child's is the one that appeared after it started
            new = set(glob.glob("/sys/class/kfd/kfd/proc/*")) - before
            files = [f for d in sorted(new) for f in glob.glob(d + "/stats_*/cu_occupancy")]
            time.sleep(0.1)
        if not files:
            print("no KFD stats for the child", flush=True)
            return 1
        def read(f):
            try:
                with open(f) as fh:
                    return int(fh.read().strip() or 0)
            except OSError:  # a short-lived GPU process (not the burn) went away
                return None

        # wait for the burn to show waves at all; keep only its file
        t0 = time.time()
        while time.time() - t0 < 60:
            new = set(glob.glob("/sys/class/kfd/kfd/proc/*")) - before
            files = [f for d in sorted(new) for f in glob.glob(d + "/stats_*/cu_occupancy")]
            live = [f for f in files if (read(f) or 0) > 0]
            if live:
                files = live
                break
            time.sleep(0.05)
        busy_files = glob.glob("/sys/class/drm/card*/device/gpu_busy_percent")
        vals, stamps, busy = [], [], []
        t0 = time.time()
        while time.time() - t0 < secs:
            vals.append(sum(read(f) or 0 for f in files))
            busy.append(read(busy_files[0]) if busy_files else None)
            stamps.append(time.time() - t0)
            time.sleep(period)
        hist = collections.Counter(vals)
        runs, cur = [], 0
        for v in vals:
            if v == 0:
                cur += 1
            elif cur:
                runs.append(cur)
                cur = 0
        if cur:
            runs.append(cur)
        print(f"files {files}")
        print(f"reads {len(vals)} over {secs} s (period {period * 1e3:.1f} ms): zero fraction "
              f"{hist.get(0, 0) / len(vals):.3f}; histogram {sorted(hist.items())}")
        print(f"zero runs (reads): n={len(runs)} max={max(runs) if runs else 0} "
              f"mean={sum(runs) / len(runs) if runs else 0:.1f}")
        print("first 80:", vals[:80], flush=True)
        print("gpu_busy_percent first 80:", busy[:80], "child alive:", child.poll() is None, flush=True)
    finally:
        child.kill()
        out, _ = child.communicate()
        print("child output:", (out or "")[-500:], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
