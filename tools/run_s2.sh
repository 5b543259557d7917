#!/bin/bash
# session script: the VQ-VAE's skinny weight gradients on a side stream -- GPU suite, then the VQ-VAE step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s33
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s33/tests.log 2>&1 || { tail -30 gpurun_out/s33/tests.log; exit 1; }
tail -1 gpurun_out/s33/tests.log
VAR=ARCWELD_SIDE_WGRAD bash tools/ab_env_bench.sh 0 1 3 || exit 1
echo done
