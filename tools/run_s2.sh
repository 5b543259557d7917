#!/bin/bash
# session script: LayerNorm backward with bf16 input gradients -- GPU suite, then the decoder step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s29
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s29/tests.log 2>&1 || { tail -30 gpurun_out/s29/tests.log; exit 1; }
tail -1 gpurun_out/s29/tests.log
VAR=ARCWELD_LN_DY_F32 ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 1 0 3 || exit 1
echo done
