#!/bin/bash
# One GPU-box pass: gpu tests, bench, rocprofv3 kernel stats of the bench. Every GPU step has its own limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -z "$SKIP_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -30 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
fi
