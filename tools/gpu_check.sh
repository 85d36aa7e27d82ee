#!/bin/bash
# GPU-box validation script (run from the repo root via gpurun).  Every GPU step has
# its own time limit; a fault/abort/timeout stops the script, test failures do not.
#   STEPS=smoke,pytest,bench,prof,pmc bash tools/gpu_check.sh
# Steps (comma list):
#   smoke      __graft_entry__.smoke()
#   pytest     the whole -m gpu suite (heartbeat file under $OUT for long cases); PYTEST_PATHS
#              narrows it (test ids, space-separated), PYTEST_ARGS adds options (no spaces inside one)
#   bench      bench.py N = 1 (rotating buffers) and its register-kernel variant
#   prof       rocprofv3 kernel trace + stats of bench.py N = 1
#   pmc        one rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) of bench.py
#   hbmsweep   tools/hbm_sweep.hip: C2 variants and calibration streams, rotating buffers
#   ipcprobe   tools/ipc_probe.hip: IPC export after free / regrowth, import capacity (N = 32 / 64)
#   rehearse   bench.py's N > 1 line with 2 / 4 ranks on GPU 0 (gloo), every leg
#   rehearse8  the same with 8 ranks (the driver's N = 8 path on one device)
#   meshprof   rank 0 of a 4 / 8-rank mesh job under rocprofv3 (trace, FETCH_SIZE, WRITE_SIZE)
#   campaign   tools/fault_campaign.sh: the reference's random-kill campaign, both schedules
#   sweep      tools/size_sweep.py with 2 / 4 / 8 ranks on GPU 0
#   e2e        host-buffer Raben end to end: chunk pipeline on / off, zero copy (1 / 2 / 4 ranks)
#   latency    tools/latency_probe.py with 2 / 4 / 8 ranks on GPU 0 (gated one-shot vs not)
#   gateprobe  tools/gate_probe.hip: the gated launch alone (latency hidden, go / skip, timeout, overtaken)
#   syncprobe  tools/sync_probe.hip: device round trip of one step
#   cpubase    tools/cpu_schedule_bench.py on this box's host cores
#   xgmi       tools/xgmi_probe.hip: one link / all peers, pull / push / copy engines (loopback on one GPU)
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
stop_on_fault() { # $1 = rc, $2 = step
    local rc=$1
    echo "$2 rc=$rc"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP after $2 (rc=$rc)"; exit "$rc"; fi
}
STEPS=${STEPS:-smoke,pytest,bench,prof}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has smoke; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if has pytest; then
  FTAR_HEARTBEAT=$OUT/heartbeat.txt timeout -k 10 ${PYTEST_TIMEOUT:-1500} python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -v \
      --timeout 900 --timeout-method thread -p no:cacheprovider -rf --durations=25 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -6 "$OUT/pytest_gpu.log"; stop_on_fault $rc pytest
fi
if has bench; then
  timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench.json"; stop_on_fault $rc bench
  timeout -k 10 300 python bench.py --variant 0 --no-cpu-baseline > "$OUT/bench_v0.json" 2>> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench_v0.json"; stop_on_fault $rc bench_v0
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_c2" -o c2 --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 100 --warmup 5 --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
  rc=$?; tail -3 "$OUT/prof_c2.log"; stop_on_fault $rc prof_c2
fi
if has pmc; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$ROOT/$OUT/pmc_$ctr" -o pmc --output-format csv -- \
        python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/pmc_$ctr.log" 2>&1
    rc=$?; tail -2 "$OUT/pmc_$ctr.log"; stop_on_fault $rc pmc_$ctr
  done
fi
if has hbmsweep; then
  timeout -k 10 180 tools/_build/hbm_sweep 40 4 > "$OUT/hbm_sweep.txt" 2>&1
  rc=$?; tail -3 "$OUT/hbm_sweep.txt"; stop_on_fault $rc hbmsweep
  timeout -k 10 180 tools/_build/hbm_sweep 40 4 f > "$OUT/hbm_sweep_focused.txt" 2>&1
  rc=$?; tail -1 "$OUT/hbm_sweep_focused.txt"; stop_on_fault $rc hbmsweep_f
fi
if has ipcprobe; then
  timeout -k 10 120 tools/_build/ipc_probe > "$OUT/ipc_probe.json" 2>&1
  rc=$?; cat "$OUT/ipc_probe.json"; stop_on_fault $rc ipcprobe
  # the capacity phase again with 128 MiB blocks: 252 imports mapping 31.5 GiB of the peer's HBM
  timeout -k 10 180 tools/_build/ipc_probe 252 128 > "$OUT/ipc_probe_128.json" 2>&1
  rc=$?; grep capacity "$OUT/ipc_probe_128.json"; stop_on_fault $rc ipcprobe_128
fi
if has rehearse || has rehearse8; then
  ns="2 4"; has rehearse8 && ns="8"
  for n in $ns; do
    FTAR_DEVICE=0 FTAR_C5_RANKS=${C5_RANKS:-5} timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps ${REH_STEPS:-5} \
        --warmup 1 --dist-backend gloo > "$OUT/rehearse_$n.json" 2> "$OUT/rehearse_$n.err" &
    pid=$!
    while kill -0 $pid 2>/dev/null; do sleep 30; echo "rehearse_$n running $(date +%T)"; done
    wait $pid; rc=$?; tail -c 600 "$OUT/rehearse_$n.json"; tail -3 "$OUT/rehearse_$n.err"; stop_on_fault $rc rehearse_$n
  done
fi
if has meshprof; then
  for p in 4 8; do
    DM=$(python3 -c "print(','.join(['0']*$p))")
    for mode in trace FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 180 fault-tolerant_amd/bin/ftrun -np $p --devmap $DM tools/rank_prof.sh "$OUT/mesh_p${p}_$mode" $mode \
          python3 tools/prof_worker.py 67108864 10 > "$OUT/mesh_p${p}_$mode.log" 2>&1
      rc=$?; stop_on_fault $rc meshprof_p${p}_$mode
    done
  done
fi
if has campaign; then
  timeout -k 10 900 tools/fault_campaign.sh "$OUT/campaign" ${CAMPAIGN_RUNS:-12} > "$OUT/campaign.log" 2>&1
  rc=$?; tail -3 "$OUT/campaign.log"; stop_on_fault $rc campaign
fi
if has sweep; then
  # per-call time over message sizes, 2 / 4 / 8 ranks sharing GPU 0
  for n in ${SWEEP_RANKS:-2 4 8}; do
    timeout -k 10 300 fault-tolerant_amd/bin/ftrun -np $n --devmap 0,0,0,0,0,0,0,0 python -u tools/size_sweep.py \
        "$OUT/sweep_$n.json" > "$OUT/sweep_$n.log" 2>&1
    rc=$?; tail -2 "$OUT/sweep_$n.log"; stop_on_fault $rc sweep_$n
  done
fi
if has e2e; then
  # host-buffer Raben end to end, chunk pipeline on / off, and the device entry point on
  # the same pinned buffers (zero copy), 1 / 2 / 4 ranks on GPU 0
  for n in 1 2 4; do for mode in pipe1 pipe0 zc; do
    hp=1; zc=0; [ $mode = pipe0 ] && hp=0; [ $mode = zc ] && zc=1
    FTAR_HOST_PIPE=$hp E2E_ZERO_COPY=$zc timeout -k 10 200 fault-tolerant_amd/bin/ftrun -np $n --devmap 0,0,0,0 \
        python -u tools/e2e_probe.py >> "$OUT/e2e.json" 2>> "$OUT/e2e.err"
    rc=$?; stop_on_fault $rc e2e_${n}_$mode
  done; done
  cat "$OUT/e2e.json"
fi
if has latency; then
  # per-call fixed cost of a 4 KiB call, ranks sharing GPU 0 (tools/latency_probe.py):
  # one-shot with its launch gated ahead of the barrier vs launched after it, mesh, RD
  for n in ${LAT_RANKS:-2 4 8}; do
    DM=$(python3 -c "print(','.join(['0']*$n))")
    timeout -k 10 180 fault-tolerant_amd/bin/ftrun -np $n --devmap $DM python -u tools/latency_probe.py \
        "$OUT/latency_${n}ranks.json" > "$OUT/latency_${n}ranks.log" 2>&1
    rc=$?; tail -c 400 "$OUT/latency_${n}ranks.log"; echo; stop_on_fault $rc latency_$n
  done
fi
if has gateprobe; then
  timeout -k 10 120 tools/_build/gate_probe > "$OUT/gate_probe.json" 2>&1
  rc=$?; cat "$OUT/gate_probe.json"; stop_on_fault $rc gateprobe
fi
if has syncprobe; then
  timeout -k 10 120 tools/_build/sync_probe > "$OUT/sync_probe.json" 2>&1
  rc=$?; cat "$OUT/sync_probe.json"; stop_on_fault $rc syncprobe
fi
if has cpubase; then
  timeout -k 10 900 python tools/cpu_schedule_bench.py --out "$OUT/cpu_schedule_bench.json" > "$OUT/cpubase.log" 2>&1
  rc=$?; tail -c 600 "$OUT/cpu_schedule_bench.json"; stop_on_fault $rc cpubase
fi
if has xgmi; then
  timeout -k 10 240 tools/_build/xgmi_probe > "$OUT/xgmi_probe.json" 2>&1
  rc=$?; cat "$OUT/xgmi_probe.json"; stop_on_fault $rc xgmi
fi
echo ALLDONE
