#!/bin/bash
# Same-box A/B of an environment switch on the VQ-VAE bench line.  usage: VAR=NAME bash tools/ab_env_bench.sh A B [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out/abenv
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --no-transformer --no-fp32 --no-stress > gpurun_out/abenv/$v$i.log 2>&1 || { tail -5 gpurun_out/abenv/$v$i.log; exit 1; }
    tail -1 gpurun_out/abenv/$v$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$VAR=$v', d['value'], d['ms_per_step'])"
  done
done
