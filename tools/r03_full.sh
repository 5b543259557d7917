#!/bin/bash
# Round-3 evidence pass on one GPU box: full GPU suite, smoke, the default bench line, the VQ-VAE kernel trace + PMC
# passes (tools/prof_round.sh) and the transformer decoder step's (tools/prof_transformer.sh).
# usage: TAG=r03_x bash tools/r03_full.sh -> gpurun_out/$TAG, gpurun_out/prof_$TAG, gpurun_out/proft_$TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_full}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
TAG=${TAG:-r03_full} EXTRA="--no-transformer" timeout -k 10 900 bash tools/prof_round.sh || exit 1
TAG=${TAG:-r03_full} timeout -k 10 900 bash tools/prof_transformer.sh || exit 1
echo done
