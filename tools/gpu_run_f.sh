# GPU box: hardware profiles of the N > 1 exchange kernels, every rank on GPU 0:
# rank 0 of a p-rank mesh job under rocprofv3 (kernel trace; FETCH_SIZE; WRITE_SIZE)
set -u
OUT=gpurun_out/F
mkdir -p $OUT
export TMPDIR=/tmp
FT=fault-tolerant_amd/bin/ftrun
for p in 4 8; do
  DM=$(python3 -c "print(','.join(['0']*$p))")
  timeout -k 10 180 $FT -np $p --devmap $DM tools/rank_prof.sh $OUT/p${p}_trace trace python3 tools/prof_worker.py 67108864 10 > $OUT/p${p}_trace.log 2>&1; rc=$?; echo "p$p trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 $FT -np $p --devmap $DM tools/rank_prof.sh $OUT/p${p}_$ctr $ctr python3 tools/prof_worker.py 67108864 10 > $OUT/p${p}_$ctr.log 2>&1; rc=$?; echo "p$p $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo ALLDONE
