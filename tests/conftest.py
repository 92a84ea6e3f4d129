import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    # torch bundles its own libamdhip64.so.7; load it before any of our HIP plugins so the
    # process ends up with one HIP runtime (see csrc/gpuexp/sentinel.hip factory comment).
    # Also initialise that runtime first when a GPU is present: measured on the box, HIP
    # initialised by our sentinel before torch (with amdsmi in the same process) makes
    # the interpreter hang at exit; torch-first is clean (profiles/provenance/tools/probe_order.sh, D vs E).
    try:
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")
    except ImportError:
        pass
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def native():
    from kubernetes_gpu_exporter_amd._native import load
    return load()


@pytest.fixture
def mock_engine(native):
    """Manual-tick mock engine (no sampler thread), HTTP on an ephemeral port."""
    engines = []

    def make(n=1, http=True, **kw):
        c = native.EngineConfig()
        c.backend = "mock"
        c.mock_devices = n
        c.interval_s = 0
        c.serve_http = http
        c.http.host = "127.0.0.1"
        c.http.port = 0
        for k, v in kw.items():
            setattr(c, k, v)
        e = native.Engine(c)
        e.start()
        engines.append(e)
        return e

    yield make
    for e in engines:
        e.stop()


@pytest.fixture
def on_gpu():
    try:
        import torch
        ok = torch.cuda.is_available()
    except Exception:
        ok = False
    if not ok:
        pytest.skip("no GPU")
    return True
