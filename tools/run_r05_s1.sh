set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_s1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_enc_chain.py -k vqvae_b1024 -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -30 $O/t.log
[ $rc -eq 0 ] || exit $rc
VAR=ARCWELD_ENC_CHAIN bash tools/ab_env_bench.sh 0 1 2
