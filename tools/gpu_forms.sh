#!/bin/bash
# The -m gpu suite under forced transport forms: every test that
# asserts a form pins it, so the suite must pass whatever the environment selects.
#   FORMS="default mesh0 push2 hostag" OUT=gpurun_out/x bash tools/gpu_forms.sh
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
for f in ${FORMS:-default mesh0 push2}; do
  case $f in
    default) envs="" ;;
    mesh0) envs="FTAR_MESH=0" ;;
    push2) envs="FTAR_PUSH=2" ;;
    unroll4) envs="FTAR_TREE_UNROLL=4" ;;
    hostag) envs="FTAR_MESH_WAIT=0" ;;
    *) echo "unknown form $f"; exit 2 ;;
  esac
  env $envs timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider -rf --durations=${DURATIONS:-30} > "$OUT/pytest_gpu_$f.log" 2>&1
  rc=$?
  echo "form $f rc=$rc: $(tail -1 "$OUT/pytest_gpu_$f.log")"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP after $f (rc=$rc)"; exit "$rc"; fi
done
