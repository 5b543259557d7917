#!/bin/bash
# Same-box A/B of the GEMM tile policy (bench --gemm-tile: 0 automatic, 256 every eligible bf16 launch on the 256-row
# ping-pong tile) on the VQ-VAE line and the pretokenized transformer line.
set -o pipefail
mkdir -p gpurun_out/abtile
for i in 1 2; do
  for t in 0 256; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-transformer --no-fp32 --no-stress --gemm-tile $t > gpurun_out/abtile/v$t$i.log 2>&1 || { tail -5 gpurun_out/abtile/v$t$i.log; exit 1; }
    timeout -k 10 300 python bench.py --only transformer_pretokenized --no-profile --gemm-tile $t > gpurun_out/abtile/t$t$i.log 2>&1 || { tail -5 gpurun_out/abtile/t$t$i.log; exit 1; }
    v=$(tail -1 gpurun_out/abtile/v$t$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")
    tr=$(tail -1 gpurun_out/abtile/t$t$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());t=d.get('transformer_pretokenized',d);print(t['value'], t['ms_per_step'])")
    echo "tile=$t vqvae $v transformer $tr"
  done
done
