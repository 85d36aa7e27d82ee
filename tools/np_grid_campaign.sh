#!/bin/bash
# The reference's fault campaign (run/run_test.sh) at its own rank counts on one GPU:
# RD at N = 12 and 16, Raben at N = 16 (the reference's campaign rows: RD N = 12 / 16,
# data/data_fault/log_single_RD.csv; Raben N = 17, log_single_Raben.csv -- a GPU box admits
# at most 16 processes on its GPU, so Raben runs at 16).  KILLS single-kill runs and NOKILL
# no-kill runs per point, every rank on GPU 0 (time-sliced).  FTAR_NP_POINTS="raben:15 ..."
# picks other points (Raben at 15 = 8 + 7 idle spares: recoveries at a large N).
#   tools/np_grid_campaign.sh OUTDIR [KILLS] [NOKILL]
set -u
OUT=$1
KILLS=${2:-10}
NOKILL=${3:-3}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export FTAR_DEVMAP=0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0
for point in ${FTAR_NP_POINTS:-rd:12 rd:16 raben:16}; do
    algo=${point%:*}
    n=${point#*:}
    for k in 1 0; do
        runs=$([ $k = 1 ] && echo $KILLS || echo $NOKILL)
        FTAR_NMIN=$n FTAR_NMAX=$n FTAR_CAMPAIGN_ALGOS=$algo FTAR_CAMPAIGN_KILLS=$k \
            timeout -k 10 600 "$ROOT/tools/fault_campaign.sh" "$OUT/n$n" "$runs" || exit $?
    done
done
