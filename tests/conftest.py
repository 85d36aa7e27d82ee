import fcntl
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer multi-process runs")
    # FTAR_HEARTBEAT=<file>: a line every 20 s naming the running test, so a long
    # full-size case is not mistaken for a hang by a watchdog that watches output files
    path = os.environ.get("FTAR_HEARTBEAT")
    if path:
        import threading
        import time

        def beat():
            while True:
                with open(path, "a") as f:
                    f.write(f"{time.strftime('%H:%M:%S')} {_current[0]}\n")
                time.sleep(20)

        threading.Thread(target=beat, daemon=True).start()


_current = ["(collecting)"]


def pytest_runtest_logstart(nodeid, location):
    _current[0] = nodeid


def load_package():
    """Import fault-tolerant_amd/ (a directory name that is not an identifier)."""
    path = os.path.join(ROOT, "fault-tolerant_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("ftar_amd", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ftar_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def hostsim():
    # one build at a time (pytest-xdist workers share the output directory)
    with open(os.path.join(ROOT, "tests", "hostsim", ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "hostsim")], check=True)
    return os.path.join(ROOT, "tests", "hostsim", "_build")


@pytest.fixture(scope="session")
def ftar():
    return load_package()


# Tests that drive the GPU from the pytest process itself (torch tensors in-process) go
# last: once this process holds a GPU context, every multi-rank job after it has one
# process more on the device than it launches, and at 8 ranks that exceeds the 8
# process slots (VMIDs) the hardware scheduler runs at once -- the job's processes are
# then time-sliced and an 8-rank case takes 2-4x longer.
IN_PROCESS_GPU = ("test_gpu_kernels.py",)


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in IN_PROCESS_GPU)
