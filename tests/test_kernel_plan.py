"""Host-side coverage check of the segment kernel's work plan (tests/kernel_plan): the
grid planner and the block -> (piece, tile) map the kernel itself calls process every
vector tile and scalar element of every segment exactly once -- interleaved, capped
and misaligned launches included.  Built with hipcc, run on the CPU."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_covers_every_unit_once():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "fault-tolerant_amd")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "kernel_plan")], check=True)
    cp = subprocess.run([os.path.join(ROOT, "tests", "kernel_plan", "_build", "plan_check"), "5000"],
                        capture_output=True, text=True, timeout=300)
    assert cp.returncode == 0, cp.stdout + cp.stderr
    assert cp.stdout.startswith("OK 5000 cases")
