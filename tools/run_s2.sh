#!/bin/bash
# session script: full GPU suite on the graph-piece refactor; an extra graph seam between the VQ-VAE forward and backward
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s21
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s21/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s21/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s21/pytest_gpu.log
VAR=ARCWELD_EXTRA_SPLIT bash tools/ab_env_bench.sh 0 1 3 || exit 1
echo done
