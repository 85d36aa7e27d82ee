#!/bin/bash
# Compare campaign: the counterpart of the reference's slurm/test_compare.slurm.  For every
# (NP, buffer size) point it runs the two fault-tolerant drivers and the two vendor
# baselines (RCCL ncclAllReduce, src/original) with ftrun, then check_compare.py appends
# the rows to ../data/data_compare/*.csv.
#   ./run_compare.sh [REPEATS]        (reference: 50 repeats, NP 4..64, 1..2^27 ints)
# One rank per GPU (RCCL refuses two ranks on one GPU), so NP defaults to 2 4 8.
#   FTAR_CMP_NPS="2 4 8"  FTAR_CMP_BUF_MIN=1  FTAR_CMP_BUF_MAX=134217728  FTAR_TIMEOUT=60
#   FTAR_CMP_BUF_MUL=2 (the size grid's factor: the reference doubles)
#   FTAR_CMP_RD / FTAR_CMP_RABEN / FTAR_CMP_ORIG_RD / FTAR_CMP_ORIG_RABEN: executables
set -u
cd "$(dirname "$0")"
OUT=${FTAR_CMP_OUT:-../out}
export FTAR_CMP_OUT=$OUT
mkdir -p "$OUT" "${FTAR_CMP_DATA:-../data/data_compare}"
REPEATS=${1:-50}
NPS=${FTAR_CMP_NPS:-"2 4 8"}
BUF_MIN=${FTAR_CMP_BUF_MIN:-1}
BUF_MAX=${FTAR_CMP_BUF_MAX:-134217728}
BUF_MUL=${FTAR_CMP_BUF_MUL:-2}
TIMEOUT=${FTAR_TIMEOUT:-60}
RD=${FTAR_CMP_RD:-../src/rd/main}
RABEN=${FTAR_CMP_RABEN:-../src/raben/main}
ORIG_RD=${FTAR_CMP_ORIG_RD:-../src/original/rd.exe}
ORIG_RABEN=${FTAR_CMP_ORIG_RABEN:-../src/original/raben.exe}

run_one() { # np size exe out
    timeout -k 10 "$TIMEOUT" ../bin/ftrun -np "$1" "$3" "$2" > "$OUT/$4.txt" 2>> "$OUT/compare_err.txt"
}

for rep in $(seq 1 "$REPEATS"); do
    echo "$rep"
    for np in $NPS; do
        buf=$BUF_MIN
        while [ "$buf" -le "$BUF_MAX" ]; do
            run_one "$np" "$buf" "$ORIG_RD" original_rd
            run_one "$np" "$buf" "$RD" rd
            run_one "$np" "$buf" "$ORIG_RABEN" original_raben
            run_one "$np" "$buf" "$RABEN" raben
            python3 ../analysis/check_compare.py
            buf=$((buf * BUF_MUL))
        done
    done
done
