#!/bin/bash
# session script: VQ forward with / without its count and squared-error atomics (probe library), isolated
set -o pipefail
export TMPDIR=/tmp
D=$PWD/vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
P1=$PWD/ablib/nocounts/libarcweld_amd.so; P2=$PWD/ablib/nosq/libarcweld_amd.so
for i in 1 2; do
  for L in $D $P1 $P2; do
    echo "== $(basename $(dirname $L))"
    ARCWELD_LIB=$L timeout -k 10 120 python tools/probe/vq_probe.py 2>&1 | grep "N 16384" || exit 1
  done
done
echo done
