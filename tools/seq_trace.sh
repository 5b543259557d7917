#!/bin/bash
# Kernel-trace CSV of a short VQ-VAE bench run (for reading the per-replay kernel sequence).
# usage: bash tools/seq_trace.sh -> gpurun_out/seq/run_kernel_trace.csv
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/seq
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/seq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-profile --no-transformer --steps 3 --warmup 2 > gpurun_out/seq/trace.log 2>&1 || { tail -20 gpurun_out/seq/trace.log; exit 1; }
find gpurun_out/seq -name '*kernel_trace.csv' -exec cp {} gpurun_out/seq/kt.csv \;
echo done
