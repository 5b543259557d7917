#!/bin/bash
# session script: decoder input-gradient layout/tile probe; LayerNorm backward look-ahead A/B; attention tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_decoder_module.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s17/att_tests.log 2>&1 || { tail -30 gpurun_out/s17/att_tests.log; exit 1; }
tail -1 gpurun_out/s17/att_tests.log
timeout -k 10 200 python tools/probe/tdgrad_probe.py 2>&1 | grep -v amdgpu.ids
VAR=AW_LN_BWD_LA ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 1 2 3 || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/s18
AW_WT_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "wgrad_batch" -x -q --timeout 240 --timeout-method thread > gpurun_out/s18/queue_tests.log 2>&1 || { tail -30 gpurun_out/s18/queue_tests.log; exit 1; }
tail -1 gpurun_out/s18/queue_tests.log
for q in 0 1 0 1; do
  echo "AW_WT_QUEUE=$q"; AW_WT_QUEUE=$q timeout -k 10 200 python tools/probe/wgrad_tt_probe.py 10 2>&1 | grep -v amdgpu.ids || exit 1
done
VAR=AW_WT_QUEUE ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 0 1 2 || exit 1
echo done
P=$PWD/ablib/lnf/libarcweld_amd.so
ARCWELD_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -k layernorm -x -q --timeout 240 --timeout-method thread > gpurun_out/s18/lnf_tests.log 2>&1 || { tail -30 gpurun_out/s18/lnf_tests.log; exit 1; }
tail -1 gpurun_out/s18/lnf_tests.log
VAR=ARCWELD_LIB ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh $PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so $P 2 || exit 1
echo done2
