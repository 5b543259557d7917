#!/bin/bash
# Same-box A/B of an environment switch on one bench line (default: the VQ-VAE configs[1] step).
# usage: VAR=NAME [ARGS="--only transformer_pretokenized"] bash tools/ab_env_bench.sh A B [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
ARGS=${ARGS:---no-cpu-baseline --no-profile --no-transformer --no-fp32 --no-stress}
mkdir -p gpurun_out/abenv
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py $ARGS --no-profile --detail "" > gpurun_out/abenv/$VAR$v$i.log 2>&1 || { tail -5 gpurun_out/abenv/$VAR$v$i.log; exit 1; }
    tail -1 gpurun_out/abenv/$VAR$v$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$VAR=$v', d['value'], d['ms_per_step'])"
  done
done
