# GPU box: bench.py paths as tests (N=1 line, 2-rank SCALE path), then the fault campaign
set -u
OUT=gpurun_out/E
mkdir -p $OUT
export FTAR_HEARTBEAT=$OUT/heartbeat.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py -v --timeout 600 --timeout-method thread -p no:cacheprovider -rA > $OUT/pytest_bench.log 2>&1; rc=$?; tail -5 $OUT/pytest_bench.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 tools/fault_campaign.sh $OUT/campaign 12 > $OUT/campaign.log 2>&1; rc=$?; tail -5 $OUT/campaign.log; echo "campaign rc=$rc"
exit $rc
