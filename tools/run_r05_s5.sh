set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_enc_chain.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -2 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe/enc_chain_probe.py 2>&1 | grep -v amdgpu.ids
VAR=ARCWELD_ENC_CHAIN_STORE bash tools/ab_env_bench.sh wt nt 2
