#!/bin/bash
# Drop-in for the reference's run/run_mpi.sh: start the job under a timeout and, in
# parallel, the random killer.
#   ./run_mpi.sh N DELAY BUF_SIZE TIMEOUT KILL_VALUE EXE_PATH
# The GPU Allreduce of one buffer takes milliseconds, so the fault-tolerant step loop is
# stretched to FTAR_LOOP_SECONDS (default 4 s, spread over its steps, busy-waiting: ranks
# stay in R state) to let a kill after DELAY = 2-3 s land in the middle of the schedule,
# as in the reference's 2-4 s CPU runs.
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
export FTAR_LOOP_SECONDS=${FTAR_LOOP_SECONDS:-4}
# The program goes through FTAR_PROG, so neither `timeout` nor the launcher has "main" on
# its command line: the killer's candidates (kill_procs.sh) are the rank processes only.
FTAR_PROG=./$EXE_PATH timeout "$TIMEOUT" ../bin/ftrun -np $N $BUF_SIZE > ../out/mpi_out.txt &
# FTAR_KILLER swaps the killer (e.g. one that only targets this job's ranks, whose
# launcher pid is exported as FTAR_JOB_PID); the default is the reference's.
FTAR_JOB_PID=$! ${FTAR_KILLER:-./kill_procs.sh} "$DELAY" "$KILL" > ../out/docker_out.txt &
wait
