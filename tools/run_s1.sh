#!/bin/bash
# session script: RCCL capture-mode fix + epilogue-prefetch library A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s14
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -x -q --timeout 240 --timeout-method thread -s > gpurun_out/s14/rccl.log 2>&1 || { tail -30 gpurun_out/s14/rccl.log; exit 1; }
tail -3 gpurun_out/s14/rccl.log
ARCWELD_LIB=$PWD/ablib/pf/libarcweld_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_vqvae_full_batch.py tests/test_decoder_module.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s14/pf_tests.log 2>&1 || { tail -30 gpurun_out/s14/pf_tests.log; exit 1; }
tail -2 gpurun_out/s14/pf_tests.log
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
P=$PWD/ablib/pf/libarcweld_amd.so
VAR=ARCWELD_LIB bash tools/ab_env_bench.sh $D $P 2 || exit 1
VAR=ARCWELD_LIB ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh $D $P 2 || exit 1
echo done
