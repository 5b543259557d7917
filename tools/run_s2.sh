#!/bin/bash
# session script: ConvT forward variants + skinny weight gradients at split-K floors 12 / 6 / 4 K steps (isolated
# probe per library), then the VQ-VAE step A/B of the 4-step floor
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s28
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
for i in 1 2; do
  for L in $D $PWD/ablib/ks6/libarcweld_amd.so $PWD/ablib/ks4/libarcweld_amd.so; do
    echo "== $(basename $(dirname $L))"
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/skinny_probe.py 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
VAR=ARCWELD_LIB bash tools/ab_env_bench.sh $D $PWD/ablib/ks4/libarcweld_amd.so 2 || exit 1
echo done
