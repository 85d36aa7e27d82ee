#!/bin/bash
# tools/devwait_ab.py with 2 / 4 / 8 ranks sharing GPU 0 (every step time-boxed; stops at
# the first failing step).   OUT=gpurun_out/x bash tools/devwait_ab.sh
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for n in ${AB_RANKS:-2 4 8}; do
    DM=$(python3 -c "print(','.join(['0'] * $n))")
    timeout -k 10 240 fault-tolerant_amd/bin/ftrun -np "$n" --devmap "$DM" python -u tools/devwait_ab.py \
        "$OUT/ab_$n.json" > "$OUT/ab_$n.log" 2>&1
    rc=$?
    echo "ranks $n rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done
