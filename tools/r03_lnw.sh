#!/bin/bash
# LayerNorm-backward waves per workgroup (AW_LN_BWD_WAVES 4 / 8): decoder GPU tests on 8, then the transformer step
# A/B on one box (alternating runs) and a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/lnw
mkdir -p $OUT
AW_LN_BWD_WAVES=8 timeout -k 10 400 python -u -m pytest tests/test_decoder_module.py tests/test_gpu_attention.py tests/test_training_regime.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_w8.log 2>&1 || { tail -30 $OUT/pytest_w8.log; exit 1; }
tail -1 $OUT/pytest_w8.log
BASE="python3 bench.py --only transformer_pretokenized"
for w in 4 8; do
  AW_LN_BWD_WAVES=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$w -o run --output-format csv -- $BASE --no-profile --steps 10 > $OUT/t$w.log 2>&1 || { tail -5 $OUT/t$w.log; exit 1; }
done
for r in 1 2 3; do
  for w in 4 8; do
    AW_LN_BWD_WAVES=$w timeout -k 10 200 $BASE > $OUT/b${w}_$r.log 2>&1 || exit 1
    echo "waves=$w run=$r $(grep -o '"ms_per_step[^,]*' $OUT/b${w}_$r.log | head -1)"
  done
done
