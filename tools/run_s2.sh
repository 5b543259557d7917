#!/bin/bash
# session script: attention forward variants (early next-tile loads; lazy rescale) -- library A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s16
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
E=$PWD/ablib/EARLY/libarcweld_amd.so
Z=$PWD/ablib/LAZY/libarcweld_amd.so
ARCWELD_LIB=$Z timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s16/lazy_tests.log 2>&1 || { tail -30 gpurun_out/s16/lazy_tests.log; exit 1; }
tail -1 gpurun_out/s16/lazy_tests.log
timeout -k 10 120 python tools/probe/sdpa_ref.py 2>&1 | grep -v amdgpu.ids
for i in 1 2; do
  for L in $D $E $Z; do
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/attn_probe.py 50 2>&1 | grep -v amdgpu.ids | tr '\n' ' '; echo " <- $(basename $(dirname $L))"
  done
done
echo done
