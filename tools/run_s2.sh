#!/bin/bash
# session script: cross-entropy forward with the target id prefetched and the target logit from registers -- GPU
# suite, kernel trace of the decoder step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s36
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s36/tests.log 2>&1 || { tail -30 gpurun_out/s36/tests.log; exit 1; }
tail -1 gpurun_out/s36/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s36/tr -o run --output-format csv -- python3 bench.py --only transformer_pretokenized --no-profile --steps 10 --warmup 3 > gpurun_out/s36/tr.log 2>&1 || { tail -20 gpurun_out/s36/tr.log; exit 1; }
find gpurun_out/s36/tr -name '*kernel_stats.csv' -exec grep -h "ce_fwd\|embed_fwd" {} \;
echo done
