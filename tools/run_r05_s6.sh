set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_s6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe/enc_chain_variants.py 2>&1 | grep -v amdgpu.ids
VAR=ARCWELD_ENC_CHAIN bash tools/ab_env_bench.sh 0 1 2
