# GPU box: focused nt-store sweep (rotating buffers), kernel parity, bench N=1 with and
# without nt stores, 4-rank rehearsal with and without nt stores
set -u
OUT=gpurun_out/C
mkdir -p $OUT
timeout -k 10 180 tools/_build/hbm_sweep 40 4 f > $OUT/hbm_sweep_f.txt 2>&1; rc=$?; cat $OUT/hbm_sweep_f.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_kernels.log 2>&1; rc=$?; tail -3 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_nt1.json 2> $OUT/bench.err; rc=$?; cat $OUT/bench_nt1.json; [ $rc -eq 0 ] || exit $rc
FTAR_NT_STORE=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_nt0.json 2>> $OUT/bench.err; rc=$?; cat $OUT/bench_nt0.json; [ $rc -eq 0 ] || exit $rc
for nt in 1 0; do
  FTAR_NT_STORE=$nt FTAR_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2952$nt bench.py --gpus 4 --steps 10 --warmup 2 --dist-backend gloo --no-c5 --no-cpu-baseline > $OUT/rehearse4_nt$nt.json 2> $OUT/rehearse4_nt$nt.err; rc=$?; head -c 1500 $OUT/rehearse4_nt$nt.json; echo; [ $rc -eq 0 ] || exit $rc
done
echo ALLDONE
