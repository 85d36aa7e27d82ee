# GPU box: the full N = 8 bench line rehearsed with 8 ranks on GPU 0 (gloo), every leg
set -u
OUT=gpurun_out/H
mkdir -p $OUT
FTAR_DEVICE=0 FTAR_C5_RANKS=5 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 5 --warmup 1 --dist-backend gloo > $OUT/rehearse8.json 2> $OUT/rehearse8.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "running $(date +%T)"; done
wait $pid; rc=$?
echo "rehearse8 rc=$rc"; tail -c 1500 $OUT/rehearse8.json; tail -5 $OUT/rehearse8.err
exit $rc
