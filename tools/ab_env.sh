#!/bin/bash
# Same-box A/B of one environment knob: alternating bench runs without (A) and with (B) the assignment.
# usage (on the GPU box): bash tools/ab_env.sh VAR=value [rounds] [extra bench args...]
set -o pipefail
KV=$1; R=${2:-2}; shift 2
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for L in A B; do
    if [ $L = B ]; then export "$KV"; else unset "${KV%%=*}"; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile "$@" > gpurun_out/ab/$L$i.log 2>&1 || exit 1
    tail -1 gpurun_out/ab/$L$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L', d['value'], d['transformer']['value'])"
  done
done
