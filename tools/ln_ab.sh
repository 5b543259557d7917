#!/bin/bash
# Transformer tests + the pretokenized decoder step: the bf16-dy LayerNorm backward.
set -o pipefail
OUT=gpurun_out/${TAG:-ln_ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py tests/test_decoder_module.py tests/test_training_regime.py tests/test_submodules.py tests/test_stress.py tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --only transformer_pretokenized --no-profile > $OUT/bench$i.log 2>&1 || { tail -20 $OUT/bench$i.log; exit 1; }
tail -1 $OUT/bench$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());t=d.get('transformer_pretokenized',d);print(t['value'], t['ms_per_step'])"
done
