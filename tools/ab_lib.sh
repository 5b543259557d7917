#!/bin/bash
# Same-box A/B of two library builds / tile policies on the VQ-VAE bench step: kernel stats + step time.
# usage: A_ENV="K=V ..." A_ARGS="--flags" B_ENV=... B_ARGS=... bash tools/ab_lib.sh -> gpurun_out/ab_lib/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab_lib
mkdir -p $OUT
BASE="python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline"
run() {  # $1 = tag, $2 = env, $3 = args, rest = command prefix
  local tag=$1 envs=$2 args=$3
  shift 3
  env $envs "$@" $BASE $args
}
for i in A B; do
  ev=${i}_ENV; ar=${i}_ARGS
  run $i "${!ev} DUMMY_AB=1" "${!ar} --no-profile --steps 10" timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d $OUT/t$i -o run --output-format csv -- > $OUT/t$i.log 2>&1 || { tail -5 $OUT/t$i.log; exit 1; }
done
for r in 1 2; do
  for i in A B; do
    ev=${i}_ENV; ar=${i}_ARGS
    run $i "${!ev} DUMMY_AB=1" "${!ar}" timeout -k 10 200 > $OUT/b${i}_$r.log 2>&1 || exit 1
    echo "$i run=$r $(grep -o '"ms_per_step[^,]*' $OUT/b${i}_$r.log | head -1)"
  done
done
