#!/bin/bash
# Fault soak on the GPU (one-off campaigns beyond the suite's defaults), every step time-boxed:
#   OUT=gpurun_out/x KILL_SEEDS=0-5 KILL2_SEEDS=0-3 PROPERTY=40 bash tools/gpu_soak.sh
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
FTAR_GPU_KILL_SEEDS=${KILL_SEEDS:-0-5} FTAR_GPU_KILL2_SEEDS=${KILL2_SEEDS:-0-3} \
FTAR_GPU_PROPERTY_EXAMPLES=${PROPERTY:-40} FTAR_GPU_WIDE=1 \
  timeout -k 10 ${SOAK_TIMEOUT:-700} python -u -m pytest -q --timeout 600 --timeout-method thread -p no:cacheprovider -rf \
  tests/test_gpu_midexchange.py tests/test_gpu_fences.py > "$OUT/pytest_gpu_soak.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu_soak.log"
exit $rc
