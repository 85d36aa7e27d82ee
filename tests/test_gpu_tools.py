"""The measurement tools bench.py runs on the node (tools/Makefile, built by build()).

tools/xgmi_probe.hip measures the fabric in bench.py's N > 1 line; on the 8-GPU node it
runs the n > 1 patterns across devices.  Here (one GPU) its self-test mode puts n
"GPUs" on device 0, so every pattern's launch geometry, segment layout and destination
check runs on every GPU test pass -- the figures are HBM figures and are not asserted.
"""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "_build", "xgmi_probe")


def _run(env_extra=None, args=()):
    env = dict(os.environ, **(env_extra or {}))
    cp = subprocess.run([PROBE, *args], capture_output=True, text=True, timeout=120, env=env)
    lines = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")]
    assert lines, cp.stdout[-1000:] + cp.stderr[-1000:]
    return cp.returncode, json.loads(lines[-1])


def test_xgmi_probe_loopback():
    rc, d = _run(args=("1", "64", "3"))
    assert rc == 0 and d["ok"] and list(d["patterns"]) == ["loopback_copy"], d


@pytest.mark.parametrize("n", [2, 3, 8])
def test_xgmi_probe_patterns_virtual(n):
    """Every pattern with n virtual GPUs: all destinations hold their sources' values
    (pull / push over one "link", both ways, copy engines, all peers at once)."""
    rc, d = _run({"XGMI_PROBE_VIRTUAL": str(n)}, ("0", "64", "3"))
    assert rc == 0 and d["ok"] and d["gpus"] == n and d["virtual_on_one_device"], d
    assert set(d["patterns"]) == {"pull1", "push1", "pull1_bidir", "push1_bidir", "sdma1_bidir", "pull_all",
                                  "push_all"}, d
    assert all(p["ok"] and p["ms"] > 0 for p in d["patterns"].values()), d


def test_gate_probe():
    """tools/gate_probe.hip drives the product's gated segment kernel alone: a gate opened
    as go copies and one opened as skip leaves the output untouched (both signal); a gate
    never opened gives up after its timeout and reports it; workgroups that find a later
    sequence in their gate word skip and report -- never a blind run, never a hang."""
    cp = subprocess.run([os.path.join(ROOT, "tools", "_build", "gate_probe")], capture_output=True, text=True,
                        timeout=120)
    lines = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")]
    assert lines, cp.stdout[-1000:] + cp.stderr[-1000:]
    d = json.loads(lines[-1])
    assert cp.returncode == 0 and d["ok"], d
    assert 90 <= d["timeout_ms"] < 2000, d
