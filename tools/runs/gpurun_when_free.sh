#!/bin/bash
# Submit ONE gpurun command, re-submitting only while gpurun reports that nothing ran
# (status=transient: no free box / back-off / box lost before the command started).
# Stops at the first call whose command actually ran (ok or fail).  Usage:
#   bash tools/runs/gpurun_when_free.sh <timeout-s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-120} + 20 ))
    continue
  fi
  exit 0
done
