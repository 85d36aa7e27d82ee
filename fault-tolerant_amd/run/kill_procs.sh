#!/bin/bash
# Drop-in for the reference's run/kill_procs.sh: after DELAY seconds, SIGKILL up to N
# random running (R-state) processes of this user whose command line contains "main".
DELAY=$1
N=$2
sleep $DELAY
for ((i = 0; i < N; i++)); do
    PIDS=($(ps -u $USER -o pid,stat,cmd | grep main | grep -v grep | awk '$2 ~ /^R/ {print $1}'))
    echo ${PIDS[@]}
    if [ "${#PIDS[@]}" -eq 0 ]; then
        echo "No more PIDs to kill. Exiting."
        exit 0
    fi
    VICTIM=${PIDS[$((RANDOM % ${#PIDS[@]}))]}
    echo "Killing PID $VICTIM"
    kill -9 "$VICTIM"
    sleep 0.5
done
