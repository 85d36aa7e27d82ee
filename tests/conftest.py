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
