#!/bin/bash
# Same-box A/B of an environment switch on the pretokenized transformer line.  usage: VAR=NAME bash tools/ab_env_tr.sh A B [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out/abtr
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python bench.py --only transformer_pretokenized --no-profile > gpurun_out/abtr/$v$i.log 2>&1 || { tail -5 gpurun_out/abtr/$v$i.log; exit 1; }
    tail -1 gpurun_out/abtr/$v$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());t=d.get('transformer_pretokenized',d);print('$VAR=$v', t['value'], t['ms_per_step'])"
  done
done
