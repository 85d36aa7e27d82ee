#!/bin/bash
# The reference's fault campaign (slurm/test_fault.slurm:14-89) on this box: for each
# schedule, RUNS runs without a kill and RUNS runs with one random kill, through the
# drop-in harness (run/run_test.sh -> run_mpi.sh -> ftrun + killer -> check_fault.py),
# N drawn from [FTAR_NMIN, FTAR_NMAX].  The killer is tests/scoped_kill.sh: the
# reference's policy (R-state processes named main) restricted to this job's processes,
# so nothing else on the machine can be hit.
#   tools/fault_campaign.sh OUTDIR [RUNS]
# FTAR_CAMPAIGN_ALGOS ("raben rd") and FTAR_CAMPAIGN_KILLS ("0 1") narrow it, e.g. the
# reference's configs[4] shape: FTAR_NMIN=9 FTAR_NMAX=9 FTAR_CAMPAIGN_ALGOS=raben FTAR_CAMPAIGN_KILLS=1.
# Writes OUTDIR/log_{nokill,single}_{RD,Raben}.csv (check_fault.py rows), one progress
# line per run on stdout.
set -u
OUT=$(realpath -m "$1")
RUNS=${2:-10}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
export FTAR_KILLER=$ROOT/tests/scoped_kill.sh
export FTAR_NMIN=${FTAR_NMIN:-5} FTAR_NMAX=${FTAR_NMAX:-8}
EXEDIR=${FTAR_EXE_DIR:-../src}  # relative to run/ (run_mpi.sh starts ./$EXE)
cd "$ROOT/fault-tolerant_amd/run"
for algo in ${FTAR_CAMPAIGN_ALGOS:-raben rd}; do
    tag=$([ $algo = raben ] && echo Raben || echo RD)
    for kill in ${FTAR_CAMPAIGN_KILLS:-0 1}; do
        name=$([ $kill = 0 ] && echo nokill || echo single)
        for ((i = 0; i < RUNS; i++)); do
            ./run_test.sh $kill "$OUT/log_${name}_${tag}.csv" $algo $EXEDIR/$algo/main > /dev/null 2>&1
            echo "$algo kill=$kill run $i: $(tail -1 "$OUT/log_${name}_${tag}.csv")"
        done
    done
done
