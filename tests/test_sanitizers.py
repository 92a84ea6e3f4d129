"""Host-side sanitizer runs of the core: CMake presets tsan / asan build the
static core + two drivers and run them:
  * gpuexp_stress: sampler 100 Hz x 8 mock GPUs, 2 HTTP loops, 4 keep-alive scrapers incl.
    gzip, control-plane churn, for 3 s;
  * gpuexp_pmc_harness: the aqlprofile plugin's read machine (pmc_rounds.cc) on 8 scripted fake
    GPUs (slow, stuck -> rescue -> release, foreign resets, another profiler, stopped counters,
    queue error), an inline-round machine and a thread-mode one at once, each with a reader."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


@pytest.mark.parametrize("preset,env", [
    ("tsan", {"TSAN_OPTIONS": "halt_on_error=1"}),
    ("asan", {"ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}),
])
def test_stress_under_sanitizer(preset, env):
    if not shutil.which("cmake") or not shutil.which("ninja"):
        pytest.skip("cmake/ninja not available")
    b = subprocess.run(f"cmake --preset {preset} -G Ninja && cmake --build --preset {preset} -j 8",
                       shell=True, cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    r = subprocess.run([os.path.join(ROOT, f"build/cmake-{preset}/gpuexp_stress"), "3", "4"],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert r.returncode == 0, out[-5000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
    assert "runtime error" not in out  # UBSan
    # the PMC read machine's invariants, at 3x slower ticks (sanitizer overhead)
    r = subprocess.run([os.path.join(ROOT, f"build/cmake-{preset}/gpuexp_pmc_harness"), "3"],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0 and out.rstrip().endswith("OK"), out[-5000:]
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
    assert "runtime error" not in out
