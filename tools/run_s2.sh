#!/bin/bash
# session script: bf16 ConvT output by default (bf16 mode), decoder fills folded, one multi-tensor input copy
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s24
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s24/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s24/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/s24/pytest_gpu.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline --detail gpurun_out/s24/detail.json > gpurun_out/s24/bench.log 2>&1 || { tail -20 gpurun_out/s24/bench.log; exit 1; }
tail -1 gpurun_out/s24/bench.log | cut -c1-300
python -c "import json;d=json.loads(open('gpurun_out/s24/bench.log').read().strip().splitlines()[-1]);print({k:v.get('ms_per_step') for k,v in d['lines'].items() if isinstance(v,dict)})"
echo done
