set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "tap3 or bf16_residual or implicit_conv3" > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -1 $O/k.log
VAR=ARCWELD_TAP3 bash tools/ab_env_bench.sh 0 1 2 || exit 1
timeout -k 10 200 python -u tools/probe/wgrad_tt_probe.py 10 > $O/wt_probe.log 2>&1 || { tail -20 $O/wt_probe.log; exit 1; }
grep -v amdgpu.ids $O/wt_probe.log
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_dp_gpu.py -x -q -s --timeout 300 --timeout-method thread > $O/dp.log 2>&1 || { tail -30 $O/dp.log; exit 1; }
grep -E "passed|failed|one-rank|largest" $O/dp.log
