# GPU box: kernel parity, bench N=1 (U4 tiles, nt stores), rocprof + PMC of it, the
# 2-rank rehearsal of the N>1 line (every key), the whole -m gpu suite
set -u
OUT=gpurun_out/D
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 tools/_build/ipc_probe > $OUT/ipc_probe.json 2>&1; rc=$?; cat $OUT/ipc_probe.json; echo "ipc rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_kernels.log 2>&1; rc=$?; tail -3 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_n1.json 2> $OUT/bench.err; rc=$?; cat $OUT/bench_n1.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $OUT/prof_c2.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc_$ctr.log 2>&1; rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
FTAR_DEVICE=0 FTAR_C5_RANKS=5 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > $OUT/rehearse2.json 2> $OUT/rehearse2.err; rc=$?; echo "rehearse rc=$rc"; [ $rc -eq 0 ] || exit $rc
export FTAR_HEARTBEAT=$OUT/heartbeat.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -p no:cacheprovider -rf > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -4 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
exit $rc
