#!/bin/bash
# gpurun with retries while the pool reports no free box (status=transient); the verdict goes to $1.
# usage: bash tools/gpr.sh <logfile> <timeout> '<command>'
log=$1; to=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  grep -q "status=transient" "$log" || break
  sleep 90
done
echo "[gpr] finished after $i attempt(s)" >> "$log"
