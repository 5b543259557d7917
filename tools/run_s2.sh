#!/bin/bash
# session script: VQ code counts in LDS by default -- GPU suite, smoke, kernel trace of the VQ-VAE step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s43
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/s43/tests.log 2>&1 || { tail -30 gpurun_out/s43/tests.log; exit 1; }
tail -1 gpurun_out/s43/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s43/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-profile --no-transformer --steps 10 --warmup 3 > gpurun_out/s43/tr.log 2>&1 || { tail -20 gpurun_out/s43/tr.log; exit 1; }
tail -1 gpurun_out/s43/tr.log | cut -c1-200
find gpurun_out/s43/tr -name '*kernel_stats.csv' -exec grep -h "vq_fwd\|head_fwd_bwd1\|head_bwd2" {} \; | cut -c1-160
echo done
