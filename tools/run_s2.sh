#!/bin/bash
# session script: head scalar sums per workgroup + rotated per-channel atomic walks (head, LayerNorm backward) --
# GPU suite, isolated probes against the unrotated build, then the VQ-VAE and decoder step A/Bs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s39
# (GPU suite: 345 passed in the first s39 call)

D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
N=$PWD/ablib/norot/libarcweld_amd.so
for i in 1 2; do
  for L in $D $N; do
    echo "== $(basename $(dirname $L))"
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/head_probe.py 20 2>&1 | grep -v amdgpu.ids | grep "bfloat16" | tr '\n' ' ' || exit 1
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/ln_probe.py 2>&1 | grep -v amdgpu.ids | grep bwd || exit 1
  done
done
VAR=ARCWELD_LIB bash tools/ab_env_bench.sh $N $D 3 || exit 1
VAR=ARCWELD_LIB ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh $N $D 2 || exit 1
echo done
