"""Transport options of the C ABI (ftar_comm_set_option / get_option), exercised through
the host-sim build of the same C sources (a one-rank comm needs no GPU)."""
import ctypes
import os

import pytest


@pytest.fixture
def solo(hostsim, monkeypatch):
    for k in ("FTAR_RELAY", "FTAR_RELAY_MIN", "FTAR_OVERLAP", "FTAR_COPY_ENGINE", "FTAR_REDUNDANCY"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("FTAR_HOSTSIM_TAG", f"opt{os.getpid()}")
    L = ctypes.CDLL(os.path.join(hostsim, "libftar_hostsim.so"))
    L.ftar_init_rank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int]
    L.ftar_comm_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
    L.ftar_comm_get_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.ftar_finalize.argtypes = [ctypes.c_void_p]
    h = ctypes.c_void_p()
    assert L.ftar_init_rank(ctypes.byref(h), f"/ftar-opt-{os.getpid()}".encode(), 0, 1, 0) == 0
    yield L, h
    L.ftar_finalize(h)


def _get(L, h, opt):
    v = ctypes.c_double()
    assert L.ftar_comm_get_option(h, opt, ctypes.byref(v)) == 0
    return v.value


def test_option_defaults_and_roundtrip(solo):
    L, h = solo
    # defaults: overlap on, relay on (4 MiB threshold), loop stretch off, copy engine off,
    # redundancy auto (2: the step-0 copy moves where a spare exists and the comm spans GPUs)
    assert [_get(L, h, o) for o in range(6)] == [1.0, 1.0, float(4 << 20), 0.0, 0.0, 2.0]
    # flag-signalled drains on, tree kernel one vector per lane and source
    assert _get(L, h, 10) == 1.0 and _get(L, h, 11) == 1.0
    assert _get(L, h, 12) == float(1 << 20)  # mid-size gates off by default
    for opt, val in ((0, 0), (1, 0), (2, 1 << 20), (3, 0.5), (4, 1), (5, 1), (5, 0), (5, 2), (10, 0), (10, 1),
                     (11, 2), (11, 4), (11, 1), (12, 16 << 20), (12, 0)):
        assert L.ftar_comm_set_option(h, opt, val) == 0
        assert _get(L, h, opt) == val


def test_option_errors(solo):
    L, h = solo
    assert L.ftar_comm_set_option(h, 99, 1) == 13       # FTAR_ERR_ARG
    assert L.ftar_comm_set_option(h, 2, -1) == 13
    assert L.ftar_comm_set_option(None, 0, 1) == 13
    assert L.ftar_comm_set_option(h, 5, 3) == 13        # redundancy: 0 never, 1 always, 2 auto
    assert L.ftar_comm_set_option(h, 11, 3) == 13       # tree unroll: 1, 2 or 4
    assert L.ftar_comm_set_option(h, 11, 2.5) == 13
    v = ctypes.c_double()
    assert L.ftar_comm_get_option(h, 99, ctypes.byref(v)) == 13


@pytest.mark.parametrize("name,value,want", [("FTAR_REDUNDANCY", v, w) for v, w in (
    ("3", "13"), ("-1", "13"), ("auto", "13"), ("on", "13"), ("", "13"), ("1x", "13"), ("0", "0"), ("1", "0"),
    ("2", "0"))] + [("FTAR_MESH", "on", "13"), ("FTAR_MESH_WAIT", "2", "13"), ("FTAR_GATE_MAX", "1M", "13"),
                    ("FTAR_GATE_MAX", "16777216", "0"), ("FTAR_LOOP_SECONDS", "1.5", "0"), ("FTAR_PUSH", "3", "13"),
                    ("FTAR_GATE_HOLD_US", "-5", "13"), ("FTAR_RELAY_MIN", "0", "0")])
def test_env_redundancy_out_of_range_is_refused(hostsim, monkeypatch, name, value, want):
    """FTAR_REDUNDANCY in the environment accepts what ftar_comm_set_option accepts (0, 1, 2):
    a typo such as 3 -- or a word such as 'auto', which atoi would have read as 0 and so turned
    the step-0 copy off -- is refused with FTAR_ERR_ARG and a message; every
    other numeric knob of the comm likewise (a range each, whole numbers unless decimal)."""
    import subprocess
    import sys
    code = ("import ctypes, os\n"
            f"L = ctypes.CDLL({os.path.join(hostsim, 'libftar_hostsim.so')!r})\n"
            "L.ftar_init_rank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_int, ctypes.c_int,"
            " ctypes.c_int]\n"
            "L.ftar_finalize.argtypes = [ctypes.c_void_p]\n"
            "h = ctypes.c_void_p()\n"
            "rc = L.ftar_init_rank(ctypes.byref(h), b'/ftar-optenv-%d' % os.getpid(), 0, 1, 0)\n"
            "print(rc)\n"
            "if rc == 0: L.ftar_finalize(h)\n")
    env = dict(os.environ, FTAR_HOSTSIM_TAG=f"optenv{os.getpid()}")
    env[name] = value
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=60)
    assert cp.stdout.strip() == want, (cp.stdout, cp.stderr)
    if want != "0":
        assert f"{name}={value} " in cp.stderr and "refused" in cp.stderr
