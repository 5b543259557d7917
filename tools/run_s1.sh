set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > $O/k.log 2>&1 || { tail -40 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 200 python -u tools/probe/wgrad_tt_probe.py 10 > $O/wt_probe.log 2>&1 || { tail -20 $O/wt_probe.log; exit 1; }
grep -v amdgpu.ids $O/wt_probe.log
