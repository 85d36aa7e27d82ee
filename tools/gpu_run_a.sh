set -u
OUT=gpurun_out/A
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err; rc=$?; echo "bench rc=$rc"; cat $OUT/bench_n1.json; [ $rc -eq 0 ] || exit $rc
FTAR_DEVICE=0 FTAR_C5_RANKS=5 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > $OUT/rehearse2.json 2> $OUT/rehearse2.err; rc=$?; echo "rehearse rc=$rc"; tail -c 3000 $OUT/rehearse2.json; tail -5 $OUT/rehearse2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > $OUT/prof_c2.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pmc_$ctr -o pmc --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc_$ctr.log 2>&1; rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo ALLDONE
