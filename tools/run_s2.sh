#!/bin/bash
# session script: epilogue store policy of the decoder step's GEMMs (NT default / write-through / plain)
set -o pipefail
export TMPDIR=/tmp
A="--no-cpu-baseline --only transformer_pretokenized"
VAR=ARCWELD_QKV_STORE ARGS="$A" bash tools/ab_env_bench.sh 0 2 2 || exit 1
VAR=ARCWELD_DEC_STORE ARGS="$A" bash tools/ab_env_bench.sh 0 2 2 || exit 1
VAR=ARCWELD_DEC_STORE ARGS="$A" bash tools/ab_env_bench.sh 0 1 2 || exit 1
echo done
VAR=ARCWELD_VQ_STORE bash tools/ab_env_bench.sh 1 2 2 || exit 1
echo done2
