#!/bin/sh
# build_id.sh abi|src -- 16 hex digits identifying a build of libftar:
#   abi  the headers every binary shares (control-block layout, C ABI): baked into
#        libftar.so, ftrun and the host-sim build, compared when a rank attaches to the
#        launcher's control block (csrc/ftar_ctrl.c) -- binaries of different headers refuse
#        to run together with one clear line
#   src  every product source: baked into libftar.so at link time (ftar_build_id()); the
#        GPU test session compares it with the tree it runs from (tests/conftest.py)
# Files in a fixed order (paths relative to fault-tolerant_amd/), so every Makefile gets
# the same digest wherever it is run from.
set -e
cd "$(dirname "$0")/.."
case "${1:-abi}" in
abi) files="../include/ftar.h $(ls csrc/*.h | LC_ALL=C sort)" ;;
src) files="../include/ftar.h $(ls csrc/* tools/ftrun.c | LC_ALL=C sort)" ;;
*) echo "usage: $0 abi|src" >&2; exit 2 ;;
esac
for f in $files; do printf '%s\n' "$f"; cat "$f"; done | sha256sum | cut -c1-16
