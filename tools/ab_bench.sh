#!/bin/bash
# Same-box A/B of two library builds: alternating bench runs (VQ-VAE line + transformer line), ARCWELD_LIB selects
# the build.  usage (on the GPU box): bash tools/ab_bench.sh <libA.so> <libB.so> [rounds]
set -o pipefail
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out/ab
for i in $(seq 1 $R); do
  for L in A B; do
    lib=$A; [ $L = B ] && lib=$B
    ARCWELD_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab/$L$i.log 2>&1 || exit 1
    tail -1 gpurun_out/ab/$L$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L', d['value'], d['transformer']['value'])"
  done
done
