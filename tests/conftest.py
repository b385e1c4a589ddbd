import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP backend, libgs_hip.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture
def debug_knob():
    """Set native test switches (csrc/include/gs/debug.h) for one test, restored afterwards:
    ``debug_knob("overlap_chain", 0)``."""
    from grayscott_amd.ops import native
    defaults = {"overlap_chain": 1, "philox_generic": 0, "ipc_emulate_us": 0,
                "ipc_system_stores": 0, "cpu_ftz": 1, "gated": 1, "gate_stamps": 0,
                "ipc_pair_same_dir": 0, "gate_mode": 0, "plan_order": 0, "plan_fill": 1}
    touched = []

    def _set(name, value, which="hip"):
        native.debug_set(name, value, which)
        touched.append((name, which))

    yield _set
    for name, which in touched:
        native.debug_set(name, defaults[name], which)


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the native libraries once per session if they are missing."""
    from grayscott_amd.ops import native
    if not os.path.exists(native.lib_path("core")) or not os.path.exists(native.lib_path("hip")):
        import subprocess
        subprocess.run(["make", "-C", ROOT, "-j8", "all"], check=True)
    yield
