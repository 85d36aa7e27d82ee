# GPU box: HBM sweep of the C2 kernel on rotating buffers, then the whole -m gpu suite
set -u
OUT=gpurun_out/B
mkdir -p $OUT
timeout -k 10 120 tools/_build/hbm_sweep 40 4 > $OUT/hbm_sweep.txt 2>&1; rc=$?; cat $OUT/hbm_sweep.txt; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
export FTAR_HEARTBEAT=$OUT/heartbeat.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -p no:cacheprovider -rf > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -15 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
exit $rc
