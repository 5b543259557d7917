#!/bin/bash
# Session 12: GPU suite on the fused small-kernel library, then the same-box step A/B against ab_base.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s12
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 900 bash tools/ab_tree.sh || exit 1
echo done
