#!/bin/bash
# session script: decoder weight gradients as one batch at the end of the backward (no collective), split graphs kept
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s20
timeout -k 10 300 python -u -m pytest tests/test_training_regime.py tests/test_decoder_module.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s20/tests1.log 2>&1 || { tail -30 gpurun_out/s20/tests1.log; exit 1; }
tail -1 gpurun_out/s20/tests1.log
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_dp_gpu.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s20/tests2.log 2>&1 || { tail -30 gpurun_out/s20/tests2.log; exit 1; }
tail -1 gpurun_out/s20/tests2.log
VAR=ARCWELD_WGRAD_MERGE ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 0 1 3 || exit 1
VAR=ARCWELD_SPLIT_GRAPHS ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 0 1 2 || exit 1
echo done
