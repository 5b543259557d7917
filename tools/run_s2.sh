#!/bin/bash
# session script: vectorised embedding forward + LDS column-slice embedding backward -- GPU suite, then the decoder
# step A/B (AW_EMBED_BWD_SLICES)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s34
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s34/tests.log 2>&1 || { tail -30 gpurun_out/s34/tests.log; exit 1; }
tail -1 gpurun_out/s34/tests.log
VAR=AW_EMBED_BWD_SLICES ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 0 1 3 || exit 1
echo done
