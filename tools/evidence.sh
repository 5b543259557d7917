#!/bin/bash
# Evidence pass on one GPU box: the GPU suite, smoke, the default bench line, the VQ-VAE kernel trace + PMC passes
# (tools/prof_round.sh) and the transformer decoder step's (tools/prof_transformer.sh).
# usage: TAG=r04_x [STAGES="tests smoke bench prof proft"] bash tools/evidence.sh
#   -> gpurun_out/$TAG/{pytest_gpu.log,smoke.log,bench.log,bench.json}, gpurun_out/prof_$TAG, gpurun_out/proft_$TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-evidence}
STAGES=${STAGES:-tests smoke bench prof proft}
OUT=gpurun_out/$TAG
mkdir -p $OUT
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if has bench; then
  timeout -k 10 500 python -u bench.py --detail $OUT/bench_detail.json ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log > $OUT/bench.json
  cat $OUT/bench.json | cut -c1-600
fi
if has prof; then
  TAG=$TAG EXTRA="--no-transformer" timeout -k 10 900 bash tools/prof_round.sh || exit 1
fi
if has proft; then
  TAG=$TAG timeout -k 10 900 bash tools/prof_transformer.sh || exit 1
fi
echo done
