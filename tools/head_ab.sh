#!/bin/bash
# Un-patch head probe, then the tests that run through the head (fused training step included).
set -o pipefail
OUT=gpurun_out/${TAG:-head_ab}
mkdir -p $OUT
timeout -k 10 200 python -u tools/probe/head_probe.py 30 > $OUT/head_probe.log 2>&1 || { cat $OUT/head_probe.log; exit 1; }
grep us $OUT/head_probe.log
if [ -z "$NOTEST" ]; then
timeout -k 10 800 python -u -m pytest tests/test_head_fused.py tests/test_vqvae_module.py tests/test_vqvae_full_batch.py tests/test_gpu_kernels.py tests/test_submodules.py tests/test_dp_gpu.py tests/test_stress.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
