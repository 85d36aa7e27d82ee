set -u
export TMPDIR=/tmp
for U in 1 2 4; do
  cp fault-tolerant_amd/lib_ab/u$U/libftar.so fault-tolerant_amd/lib/libftar.so || exit 3
  for p in 4 8; do
    DM=$(python3 -c "print(','.join(['0']*$p))")
    timeout -k 10 120 fault-tolerant_amd/bin/ftrun -np $p --devmap $DM tools/rank_prof.sh gpurun_out/ab/u${U}_p$p trace \
        python3 tools/prof_worker.py 67108864 20 > gpurun_out/ab/u${U}_p$p.log 2>&1
    rc=$?; echo "u$U p$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
