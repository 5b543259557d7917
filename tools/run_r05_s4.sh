set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_s4; mkdir -p $O
timeout -k 10 120 python -u tools/debug/enc_chain_diff.py 2>&1 | grep -v amdgpu.ids | tail -4
timeout -k 10 300 python -u -m pytest tests/test_enc_chain.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe/enc_chain_variants.py 2>&1 | grep -v amdgpu.ids
EC_STORE_POLICY=0 timeout -k 10 200 python -u tools/probe/enc_chain_variants.py 2>&1 | grep -v amdgpu.ids | grep -v "stamps\|epilogue\|barrier"
timeout -k 10 120 python -u tools/probe/enc_chain_probe.py 2>&1 | grep -v amdgpu.ids
VAR=ARCWELD_ENC_CHAIN bash tools/ab_env_bench.sh 0 1 2
