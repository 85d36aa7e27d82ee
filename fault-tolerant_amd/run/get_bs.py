"""Buffer-size range for one randomised test (reference run/get_bs.py): prints MIN MAX.

The reference sizes the buffer so a CPU run lasts 2-4 s; on MI355X the Allreduce of even
the largest host buffer takes milliseconds and the run length is set by
FTAR_LOOP_SECONDS instead (run_mpi.sh), so the range only has to keep every rank's
host buffers, H2D/D2H copies and checksum loop modest: about 1.04e9 / (N + 6) int32
elements scaled to a 0.18-0.22 band, as the reference does, capped at 2^26 elements.
"""
import sys


def buffer_range(n: int):
    k = n + 6
    if 16 <= n <= 64:
        k -= 5
    mid = min(1.04e9 / k * 0.1, float(1 << 26))
    return int(mid * 1.8), int(mid * 2.2)


if __name__ == "__main__":
    import os
    lo, hi = buffer_range(int(sys.argv[1]))
    cap = int(os.environ.get("FTAR_BUF_MAX", "0"))  # e.g. small buffers for the CPU tests
    if cap:
        lo, hi = min(lo, cap // 2), min(hi, cap)
    print(lo, hi)
