set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s6
mkdir -p $O
timeout -k 10 200 python -u tools/probe/wgrad_tt_probe.py 10 > $O/wt_probe.log 2>&1 || { tail -20 $O/wt_probe.log; exit 1; }
grep -v amdgpu.ids $O/wt_probe.log
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_dp_gpu.py -x -q -s --timeout 300 --timeout-method thread > $O/dp.log 2>&1 || { tail -30 $O/dp.log; exit 1; }
grep -E "passed|failed|one-rank|largest" $O/dp.log
