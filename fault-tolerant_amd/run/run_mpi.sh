#!/bin/bash
# Drop-in for the reference's run/run_mpi.sh: start the job under a timeout and, in
# parallel, the random killer.
#   ./run_mpi.sh N DELAY BUF_SIZE TIMEOUT KILL_VALUE EXE_PATH
# The GPU Allreduce of one buffer takes milliseconds, so each tolerant barrier is
# stretched by FTAR_STEP_DELAY_MS (default 400 ms, busy-waiting: ranks stay in R state)
# to keep the run a few seconds long and let the kill land in the middle of the schedule.
N=$1
DELAY=$2
BUF_SIZE=$3
TIMEOUT=$4
KILL_VALUE=$5
EXE_PATH=$6
if [[ "$KILL_VALUE" == "0" ]]; then
    echo "Kill not enabled"
    KILL=0
elif [[ "$KILL_VALUE" == "1" ]]; then
    echo "Single Kill enabled"
    KILL=1
else
    echo "Multiple Kill enabled"
    KILL=$((RANDOM % (N - 1) + 1))
fi
export FTAR_STEP_DELAY_MS=${FTAR_STEP_DELAY_MS:-400}
timeout "$TIMEOUT" ../bin/ftrun -np $N ./$EXE_PATH $BUF_SIZE > ../out/mpi_out.txt &
./kill_procs.sh "$DELAY" "$KILL" > ../out/docker_out.txt &
wait
