#!/bin/bash
# One rank of an ftrun job under rocprofv3, the others plain:
#   ftrun -np P --devmap ... tools/rank_prof.sh <outdir> <mode> prog [args...]
# mode: trace (kernel trace + stats) or a PMC counter name (one counter per pass).
# Rank FTAR_PROF_RANK (default 0) is profiled.  bash execs rocprofv3 before anything
# touched the GPU, and rocprofv3 runs the program itself after `--`.
OUT=$1
MODE=$2
shift 2
if [ "${FTAR_RANK:-0}" = "${FTAR_PROF_RANK:-0}" ]; then
    if [ "$MODE" = trace ]; then
        exec rocprofv3 --kernel-trace --stats -d "$OUT" -o "rank$FTAR_RANK" --output-format csv -- "$@"
    else
        exec rocprofv3 --pmc "$MODE" -d "$OUT" -o "rank$FTAR_RANK" --output-format csv -- "$@"
    fi
fi
exec "$@"
