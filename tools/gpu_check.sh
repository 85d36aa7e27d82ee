#!/bin/bash
# GPU-box validation script (run from the repo root via gpurun).  Every GPU step has
# its own time limit; a fault/abort/timeout stops the script, test failures do not.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ROOT=$(pwd)
stop_on_fault() { # $1 = rc, $2 = step
    local rc=$1
    echo "$2 rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP after $2 (rc=$rc)"; exit "$rc"; fi
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *pytest* ]]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-1200} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -15 "$OUT/pytest_gpu.log"; stop_on_fault $rc pytest
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench.json"; stop_on_fault $rc bench
  timeout -k 10 300 python bench.py --variant 0 --no-cpu-baseline > "$OUT/bench_v0.json" 2>> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench_v0.json"; stop_on_fault $rc bench_v0
fi
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_c2" -o c2 --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 100 --warmup 5 --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_c2.log"; stop_on_fault $rc prof_c2
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr -d "$ROOT/$OUT/pmc_$ctr" -o pmc --output-format csv -- \
        python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/pmc_$ctr.log" 2>&1
    rc=$?; tail -2 "$OUT/pmc_$ctr.log"; stop_on_fault $rc pmc_$ctr
  done
fi
if [[ $STEPS == *rehearse* ]]; then
  # multi-rank bench path with every rank on GPU 0 (gloo for the torch side)
  for n in 2 4; do
    FTAR_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps ${REH_STEPS:-5} \
        --warmup 1 --dist-backend gloo > "$OUT/rehearse_$n.json" 2> "$OUT/rehearse_$n.err"
    rc=$?; cat "$OUT/rehearse_$n.json"; tail -3 "$OUT/rehearse_$n.err"; stop_on_fault $rc rehearse_$n
  done
fi
if [[ $STEPS == *sweep* ]]; then
  # per-call time over message sizes, 2 / 4 / 8 ranks sharing GPU 0
  for n in ${SWEEP_RANKS:-2 4 8}; do
    timeout -k 10 300 fault-tolerant_amd/bin/ftrun -np $n --devmap 0,0,0,0,0,0,0,0 python -u tools/size_sweep.py \
        "$OUT/sweep_$n.json" > "$OUT/sweep_$n.log" 2>&1
    rc=$?; tail -2 "$OUT/sweep_$n.log"; stop_on_fault $rc sweep_$n
  done
fi
if [[ $STEPS == *e2e* ]]; then
  # host-buffer Raben end to end, chunk pipeline on / off, 1 / 2 ranks on GPU 0
  for n in 2 4; do for hp in 1 0; do
    FTAR_HOST_PIPE=$hp timeout -k 10 200 fault-tolerant_amd/bin/ftrun -np $n --devmap 0,0,0,0 python -u tools/e2e_probe.py \
        >> "$OUT/e2e.json" 2>> "$OUT/e2e.err"
    rc=$?; stop_on_fault $rc e2e_${n}_$hp
  done; done
  cat "$OUT/e2e.json"
fi
if [[ $STEPS == *syncprobe* ]]; then
  # device round trip of one step: kernel + marker event + host spin (tools/sync_probe.hip)
  timeout -k 10 120 tools/_build/sync_probe > "$OUT/sync_probe.json" 2>&1
  rc=$?; cat "$OUT/sync_probe.json"; stop_on_fault $rc syncprobe
fi
if [[ $STEPS == *cpubase* ]]; then
  # CPU baseline of the schedules on this box's host cores (no GPU involved)
  timeout -k 10 900 python tools/cpu_schedule_bench.py --out "$OUT/cpu_schedule_bench.json" > "$OUT/cpubase.log" 2>&1
  rc=$?; tail -c 600 "$OUT/cpu_schedule_bench.json"; stop_on_fault $rc cpubase
fi
echo ALLDONE
