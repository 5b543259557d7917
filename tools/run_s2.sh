#!/bin/bash
# session script: no mid-backward cut without a collective (one graph piece per step) -- graph tests, then the
# VQ-VAE and decoder step A/Bs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s32
VAR=ARCWELD_MID_CUT bash tools/ab_env_bench.sh 1 0 3 || exit 1
VAR=ARCWELD_MID_CUT ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 1 0 3 || exit 1
echo done
