#!/bin/bash
# session script: attention outputs stored as whole rows through LDS (library A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s15
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
P=$PWD/ablib/att/libarcweld_amd.so
ARCWELD_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_decoder_module.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s15/att_tests.log 2>&1 || { tail -30 gpurun_out/s15/att_tests.log; exit 1; }
tail -1 gpurun_out/s15/att_tests.log
for i in 1 2; do
  for L in $D $P; do
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/attn_probe.py 50 2>&1 | tr '\n' ' '; echo " <- $(basename $(dirname $L))"
  done
done
VAR=ARCWELD_LIB ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh $D $P 2 || exit 1
echo done
