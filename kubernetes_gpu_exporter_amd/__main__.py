"""`python -m kubernetes_gpu_exporter_amd [flags]` — run the exporter."""
import sys

from .config import load_config
from .exporter import Exporter
from .utils import logfmt


def main(argv=None) -> int:
    cfg = load_config(argv)
    logfmt.setup(cfg.log_level, cfg.log_format)  # same record format as the C++ core
    return Exporter(cfg).run_forever()


if __name__ == "__main__":
    rc = main()
    # The engine is fully stopped (sampler joined, HTTP closed, sentinel drained, amdsmi
    # shut down).  Skip interpreter/static teardown: HIP and amdsmi runtime destructors
    # can block process exit, and a DaemonSet pod must terminate within its grace period.
    sys.stdout.flush()
    sys.stderr.flush()
    import os
    os._exit(rc)
