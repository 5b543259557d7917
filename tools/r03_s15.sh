#!/bin/bash
# Session 15: decoder GPU tests on the padded lm_head / fused logits-gradient path, then the transformer step A/B
# against ab_base (the previous commit).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/s15
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
AB_BASE_CMD="python3 bench.py --only transformer_pretokenized" timeout -k 10 900 bash tools/ab_tree.sh || exit 1
echo done
