#!/bin/bash
# session script: attention tests on the new forward + the decoder input-gradient layout/tile probe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py tests/test_decoder_module.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s17/att_tests.log 2>&1 || { tail -30 gpurun_out/s17/att_tests.log; exit 1; }
tail -1 gpurun_out/s17/att_tests.log
timeout -k 10 200 python tools/probe/tdgrad_probe.py 2>&1 | grep -v amdgpu.ids
echo done
