#!/bin/bash
# session script: the default bench line on the final library
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s44
timeout -k 10 500 python -u bench.py --detail gpurun_out/s44/bench_detail.json > gpurun_out/s44/bench.log 2>&1 || { tail -30 gpurun_out/s44/bench.log; exit 1; }
tail -1 gpurun_out/s44/bench.log > gpurun_out/s44/bench.json
cut -c1-400 gpurun_out/s44/bench.json
echo done
