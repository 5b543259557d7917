#!/bin/bash
# session script: non-temporal output stores in the LayerNorm and attention kernels (probe libraries, A/B)
set -o pipefail
export TMPDIR=/tmp
A="--no-cpu-baseline --only transformer_pretokenized"
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
VAR=ARCWELD_LIB ARGS="$A" bash tools/ab_env_bench.sh $D $PWD/ablib/lnnt/libarcweld_amd.so 3 || exit 1
VAR=ARCWELD_LIB ARGS="$A" bash tools/ab_env_bench.sh $D $PWD/ablib/attnt/libarcweld_amd.so 3 || exit 1
echo done
