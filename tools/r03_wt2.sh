#!/bin/bash
# A/B of the write-through variants (GEMM only / GEMM + RAdam + head) against the library, and the transformer
# grouped weight-gradient probe under the library and the split-K-8 build.
set -o pipefail
mkdir -p gpurun_out/wt2
L=vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so
W1=tools/probe/build/libarcweld_wt.so
W2=tools/probe/build/libarcweld_wt2.so
timeout -k 10 120 python -u tools/probe/twgrad_probe.py > gpurun_out/wt2/tw_lib.log 2>&1 || exit 1
ARCWELD_LIB=tools/probe/build/libarcweld_ms8.so timeout -k 10 120 python -u tools/probe/twgrad_probe.py > gpurun_out/wt2/tw_ms8.log 2>&1 || exit 1
for i in 1 2; do
  for pair in "A $L" "W1 $W1" "W2 $W2"; do
    set -- $pair
    ARCWELD_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --no-stress --no-fp32 > gpurun_out/wt2/$1_$i.log 2>&1 || exit 1
    tail -1 gpurun_out/wt2/$1_$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$1', d['value'], d['transformer']['value'])"
  done
done
