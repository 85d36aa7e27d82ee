#!/bin/bash
# Drop-in for the reference's run/run_test.sh: one randomised fault-injection test.
#   ./run_test.sh <kill 0|1|2> <log.csv> <rd|raben> <executable>
# e.g. ./run_test.sh 1 ../log/sample.csv raben ../src/raben/main
# Differences: ranks are started by ../bin/ftrun (one process per rank, rank r on GPU
# r % ngpus) instead of `singularity exec ... mpiexec --with-ft ulfm`, and N's range can
# be narrowed with FTAR_NMIN/FTAR_NMAX (default 4..32 as in the reference).
if [[ $# -ne 4 ]]; then
    echo "Usage: $0 MULTIPLE_KILL LOG_FILE ALLREDUCE_TYPE EXECUTABLE_FILE"
    exit 1
fi
mkdir -p ../out ../log
MULTIPLE_KILL=$1
LOG_FILE=$2
ALLREDUCE_TYPE=$3
EXE=$4
NMIN=${FTAR_NMIN:-4}
NMAX=${FTAR_NMAX:-32}
N=$((RANDOM % (NMAX - NMIN + 1) + NMIN))
DELAY=$((RANDOM % (3 - 2 + 1) + 2))
read MIN MAX <<< $(python3 get_bs.py $N)
BUF_SIZE=$((RANDOM % (MAX - MIN + 1) + MIN))
TIMEOUT=${FTAR_TIMEOUT:-30}
{
    echo "Generated values:"
    echo "N = $N"
    echo "DELAY = $DELAY"
    echo "BUF_SIZE = $BUF_SIZE"
    echo "TIMEOUT = $TIMEOUT"
} > ../out/test_log.txt
{ time ./run_mpi.sh $N $DELAY $BUF_SIZE $TIMEOUT "$MULTIPLE_KILL" $EXE; } >> ../out/test_log.txt 2>&1
python3 ../analysis/check_fault.py "$ALLREDUCE_TYPE" "$LOG_FILE"
rm -f ../out/mpi_out.txt ../out/docker_out.txt ../out/test_log.txt
sleep 1
