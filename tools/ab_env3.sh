#!/bin/bash
# Kernel-stats A/B/C of env / library variants on the VQ-VAE bench step (rocprofv3 kernel trace, one run each).
# usage: V1="K=V ..." V2=... V3=... bash tools/ab_env3.sh -> gpurun_out/ab_env3/t{1,2,3}/run_kernel_stats.csv
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab_env3
mkdir -p $OUT
for i in 1 2 3; do
  ev=V$i
  [ -z "${!ev+x}" ] && continue
  env ${!ev} DUMMY_AB=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- \
    python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline --no-profile --steps 10 \
    > $OUT/t$i.log 2>&1 || { tail -5 $OUT/t$i.log; exit 1; }
  echo "$i: $(grep -o '"ms_per_step[^,]*' $OUT/t$i.log | head -1)"
done
