#!/bin/bash
# Round-3 GPU pass: the new tests first, the full GPU suite, the bench line, kernel trace of the VQ-VAE bench,
# the transformer profile.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_s1}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k wgrad_conv3 -m gpu > $OUT/pytest_wgrad.log 2>&1 || { tail -40 $OUT/pytest_wgrad.log; exit 1; }
tail -3 $OUT/pytest_wgrad.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-transformer --no-profile --steps 10 --warmup 3 > $OUT/vq_bench.log 2>&1 || { tail -30 $OUT/vq_bench.log; exit 1; }
tail -1 $OUT/vq_bench.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_submodules.py tests/test_operands.py tests/test_dp_gpu.py tests/test_stress.py -m gpu > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
TAG=${TAG:-r03_s1} timeout -k 10 900 bash tools/prof_transformer.sh || exit 1
echo done
