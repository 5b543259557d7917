#!/bin/bash
# Attention kernels: GPU parity tests, then the probe at the bench shape over the A/B knobs.
# CFGS: space-separated ring,order,probe triples.
set -o pipefail
OUT=gpurun_out/${TAG:-attn_ab}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_submodules.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
for cfg in ${CFGS:-0,0,0 7,0,0 0,1,0 7,1,0}; do
  IFS=, read -r a b c <<< "$cfg"
  AW_ATTN_RING=$a AW_ATTN_ORDER=$b AW_ATTN_PROBE=$c timeout -k 10 120 python -u tools/probe/attn_probe.py 50 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
  echo "ring=$a order=$b probe=$c $(grep us $OUT/probe.log | tr '\n' ' ')"
done
