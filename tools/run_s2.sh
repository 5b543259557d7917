#!/bin/bash
# session script: the update captured into the last forward/backward graph piece -- GPU suite, then the VQ-VAE and
# decoder step A/Bs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s31
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s31/tests.log 2>&1 || { tail -30 gpurun_out/s31/tests.log; exit 1; }
tail -1 gpurun_out/s31/tests.log
VAR=ARCWELD_FUSE_UPDATE bash tools/ab_env_bench.sh 0 1 3 || exit 1
VAR=ARCWELD_FUSE_UPDATE ARGS="--no-cpu-baseline --only transformer_pretokenized" bash tools/ab_env_bench.sh 0 1 3 || exit 1
echo done
