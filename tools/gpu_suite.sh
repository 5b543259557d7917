#!/bin/bash
# Full GPU test suite, then the attention probe.  usage: TAG=x bash tools/gpu_suite.sh
set -o pipefail
OUT=gpurun_out/${TAG:-suite}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u tools/probe/attn_probe.py 50 > $OUT/attn_probe.log 2>&1 || { cat $OUT/attn_probe.log; exit 1; }
grep us $OUT/attn_probe.log
