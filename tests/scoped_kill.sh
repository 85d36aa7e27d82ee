#!/bin/bash
# Test-side replacement of run/kill_procs.sh: same policy (after DELAY s, SIGKILL up to N
# random R-state processes whose command line contains "main"), but only among the
# descendants of $FTAR_JOB_PID, so a test can never hit an unrelated process.
DELAY=$1
N=$2
sleep "$DELAY"
descendants() {
    ps -e -o pid=,ppid=,stat=,comm= | awk -v root="$FTAR_JOB_PID" '
        { pid[NR]=$1; ppid[NR]=$2; st[NR]=$3; cmd[NR]=$4 }
        END { keep[root]=1; changed=1
              while (changed) { changed=0
                  for (i=1;i<=NR;i++) if (!(pid[i] in keep) && (ppid[i] in keep)) { keep[pid[i]]=1; changed=1 } }
              for (i=1;i<=NR;i++) if (pid[i]!=root && (pid[i] in keep) && st[i] ~ /^R/ && cmd[i] == "main") print pid[i] }'
}
for ((i = 0; i < N; i++)); do
    PIDS=($(descendants))
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
