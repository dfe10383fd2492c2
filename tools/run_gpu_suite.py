"""Run the GPU test suite in this process with a native crash tracer installed (tools/abort_trace.c):
a crash after the interpreter has finalized -- in a runtime's exit-time teardown -- still prints a
backtrace.  It also reports, per test, the shared libraries a test made the process load (first
appearance in /proc/self/maps), and at exit the native objects the package still holds.

    python tools/run_gpu_suite.py [pytest args...]
"""
import atexit
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ctypes.CDLL(os.path.join(HERE, "libabort_trace.so"))
sys.path.insert(0, os.path.dirname(HERE))

import pytest  # noqa: E402


def _libs() -> set:
    out = set()
    with open("/proc/self/maps") as fh:
        for line in fh:
            parts = line.split()
            if len(parts) >= 6 and ".so" in parts[5]:
                out.add(parts[5])
    return out


class LibWatch:
    def __init__(self):
        self.seen = _libs()

    @pytest.hookimpl(hookwrapper=True)
    def pytest_runtest_protocol(self, item, nextitem):
        yield
        now = _libs()
        new = sorted(now - self.seen)
        if new:
            print(f"\n[run_gpu_suite] {item.nodeid} loaded: {' '.join(os.path.basename(p) for p in new)}", flush=True)
        self.seen = now


def _live_report() -> None:
    try:
        from audiorenderingv2_amd import renderer

        attr = {"stream": "_s", "buffer": "ptr", "group": "_g", "renderer": "_h"}
        open_ = {k: sum(1 for o in v if getattr(o, attr[k], None)) for k, v in renderer._LIVE.items()}
        print("[run_gpu_suite] tracked / still open at exit:", {k: len(v) for k, v in renderer._LIVE.items()}, open_,
              flush=True)
    except Exception as e:  # noqa: BLE001
        print("[run_gpu_suite] live report failed:", e, flush=True)
    smi = sorted(p for p in _libs() if "smi" in os.path.basename(p) or "drm" in os.path.basename(p))
    print("[run_gpu_suite] smi/drm libraries mapped at exit:", smi, flush=True)


atexit.register(_live_report)  # runs after the package's own release hook (LIFO)
sys.exit(pytest.main(sys.argv[1:], plugins=[LibWatch()]))
