#!/bin/bash
# Transformer decoder tests + its pretokenized step, then the kernel trace of that step (CE / embedding kernels).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tr_small}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_decoder_module.py tests/test_training_regime.py tests/test_submodules.py tests/test_stress.py tests/test_entry_scripts.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --only transformer_pretokenized --no-profile > $OUT/bench$i.log 2>&1 || { tail -20 $OUT/bench$i.log; exit 1; }
tail -1 $OUT/bench$i.log | python -c "import json,sys;d=json.loads(sys.stdin.read());t=d.get('transformer_pretokenized',d);print(t['value'], t['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --only transformer_pretokenized --no-profile --steps 10 --warmup 3 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
grep -E "ce_fwd|embed_bwd" $OUT/trace/run_kernel_stats.csv | cut -c1-160
