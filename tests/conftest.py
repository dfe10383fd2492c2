import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def world_scene(scene, listener, yaw=0.0):
    """Static scene + placed receiver halves, in the global-id order the engine uses
    (scene, receiver_left, receiver_right: placeReceiver, OptixModel.cpp:153-157)."""
    from audiorenderingv2_amd import place_receiver_vertices, receiver_local

    L, R = receiver_local()
    Lw = place_receiver_vertices(L.reshape(-1, 3), listener, yaw).reshape(-1, 9)
    Rw = place_receiver_vertices(R.reshape(-1, 3), listener, yaw).reshape(-1, 9)
    tv = np.concatenate([scene.tri_v, Lw, Rw]).astype(np.float32)
    ta = np.concatenate([scene.tri_abs, np.full(len(Lw), -1.0, np.float32),
                         np.full(len(Rw), -2.0, np.float32)]).astype(np.float32)
    return tv, ta


def oracle_threads() -> int:
    """Threads for the CPU oracle: the CPUs this process may run on, capped by a cgroup CPU quota (the
    GPU box's affinity mask lists the whole machine while its share is 16 CPUs)."""
    import math

    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 64))


@pytest.fixture(scope="session")
def c1_scene():
    from audiorenderingv2_amd.scene import reference_config_materials, test_obj_scene

    return test_obj_scene(reference_config_materials())


@pytest.fixture(scope="session")
def conference():
    from audiorenderingv2_amd.scene import conference_standin

    return conference_standin()


@pytest.fixture(autouse=True)
def _no_second_hip_runtime(request):
    """GPU tests must not bring another GPU framework into the test process: torch's bundled HIP
    runtime loads libamd_smi, whose global tables interpose those of RCCL's librocm_smi64; both
    libraries then destroy the same objects at interpreter exit and the process aborts (double
    free) after every test has passed (profiles/r04/exit_abort_backtrace.txt).  Device memory for a
    test comes from audiorenderingv2_amd.DeviceBuffer; torch runs only in subprocesses."""
    yield
    if request.node.get_closest_marker("gpu") is not None:
        assert "torch" not in sys.modules, f"{request.node.nodeid} imported torch into the GPU test process"


def pytest_unconfigure(config):
    # marks the end of the session in GPU logs: anything after it (a crash at interpreter exit) is
    # teardown, not a test
    print("\n[conftest] pytest session unconfigured", flush=True)
