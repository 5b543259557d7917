#!/bin/bash
# Same-box A/B of an environment switch on one bench line (default: the VQ-VAE configs[1] step).
# usage: VAR=NAME [ARGS="--only transformer_pretokenized"] bash tools/ab_env_bench.sh A B [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
ARGS=${ARGS:---no-cpu-baseline --no-profile --no-transformer --no-fp32 --no-stress}
mkdir -p gpurun_out/abenv
for i in $(seq 1 $R); do
  for t in A B; do
    [ $t = A ] && v=$A || v=$B
    log=gpurun_out/abenv/$VAR-$t$i.log
    env $VAR=$v timeout -k 10 200 python bench.py $ARGS --no-profile --detail "" > $log 2>&1 || { tail -5 $log; exit 1; }
    tail -1 $log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$VAR=$t', d['value'], d['ms_per_step'])"
  done
done
