#!/bin/bash
# Same-box A/B of two source trees (A = ./ab_base: an older commit with its own prebuilt library, B = this tree) on
# the VQ-VAE bench step: kernel trace + stats of each, then alternating timed runs.
# usage: [AB_BASE_CMD="python3 bench.py --only transformer_pretokenized"] bash tools/ab_tree.sh -> gpurun_out/ab_tree/
set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/ab_tree
mkdir -p $OUT
BASE=${AB_BASE_CMD:-"python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline"}
for i in A B; do
  d=$PWD; [ $i = A ] && d=$PWD/ab_base
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- $BASE --no-profile --steps 10 > $OUT/t$i.log 2>&1) || { tail -5 $OUT/t$i.log; exit 1; }
done
for r in 1 2 3; do
  for i in A B; do
    d=$PWD; [ $i = A ] && d=$PWD/ab_base
    (cd $d && timeout -k 10 200 $BASE > $OUT/b${i}_$r.log 2>&1) || exit 1
    echo "$i run=$r $(grep -o '"ms_per_step[^,]*' $OUT/b${i}_$r.log | head -1)"
  done
done
