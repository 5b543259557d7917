#!/bin/bash
# Persistent-grid probe (AW_GEMM_PERSIST): full-size VQ-VAE parity on it, then same-box step A/B of grids.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/persist
mkdir -p $OUT
AW_GEMM_PERSIST=256 timeout -k 10 300 python -u -m pytest tests/test_vqvae_full_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_p256.log 2>&1 || { tail -30 $OUT/pytest_p256.log; exit 1; }
tail -1 $OUT/pytest_p256.log
BASE="python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline"
for i in 0 256 384; do
  AW_GEMM_PERSIST=$i timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- $BASE --no-profile --steps 10 > $OUT/t$i.log 2>&1 || { tail -5 $OUT/t$i.log; exit 1; }
done
for r in 1 2; do
  for i in 0 256 384; do
    AW_GEMM_PERSIST=$i timeout -k 10 200 $BASE > $OUT/b${i}_$r.log 2>&1 || exit 1
    echo "persist=$i run=$r $(grep -o '"ms_per_step[^,]*' $OUT/b${i}_$r.log | head -1)"
  done
done
