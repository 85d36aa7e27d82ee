import fcntl
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_sessionstart(session):
    # host-sim segments a killed or timed-out earlier run left in /dev/shm (their owner pids
    # are dead): removed before the suite, so it does not start short of memory
    import harness
    harness.reap_shm()


def library_build_id(path=None):
    """The 'ftar-build abi=... src=...' string baked into a built libftar.so (read from the file:
    loading the library is not needed)."""
    import re
    path = path or os.path.join(ROOT, "fault-tolerant_amd", "lib", "libftar.so")
    m = re.search(rb"ftar-build abi=[0-9a-f]{16} src=[0-9a-f]{16}", open(path, "rb").read())
    return m.group(0).decode() if m else None


def tree_src_id():
    return subprocess.run([os.path.join(ROOT, "fault-tolerant_amd", "tools", "build_id.sh"), "src"],
                          capture_output=True, text=True, check=True).stdout.strip()


def pytest_collection_finish(session):
    # A GPU session runs the libraries built in this tree before it was pushed: a library
    # linked from other sources than the tree's (a stale build) would make every result
    # evidence about some other code -- refuse to start instead
    if not any(it.get_closest_marker("gpu") for it in session.items):
        return
    try:
        got, want = library_build_id(), tree_src_id()
    except OSError as e:
        pytest.exit(f"GPU session: cannot read lib/libftar.so's build id ({e}); build first (make)", returncode=3)
    if not got or not got.endswith("src=" + want):
        pytest.exit(f"GPU session: lib/libftar.so is '{got}' but the tree's sources are src={want}: "
                    "stale build, rebuild (python -c 'import __graft_entry__ as g; g.build()')", returncode=3)
    print(f"\nGPU session: {got} (the tree's sources)")


def pytest_sessionfinish(session, exitstatus):
    import harness
    harness.reap_shm()


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
