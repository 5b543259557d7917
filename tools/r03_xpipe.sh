#!/bin/bash
# XPIPE A/B: GPU suite on the variant library, K-sweep of both, same-box step A/B (tools/ab_lib.sh).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/xpipe
mkdir -p $OUT
LX=$PWD/vq-vae-transformer-arc-welding_amd/lib_x/libarcweld_amd.so
ARCWELD_LIB=$LX timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_x.log 2>&1 || { tail -30 $OUT/pytest_x.log; exit 1; }
tail -2 $OUT/pytest_x.log
timeout -k 10 120 python -u tools/probe/gemm_k_sweep.py > $OUT/ksweep_A.log 2>&1 || exit 1
ARCWELD_LIB=$LX timeout -k 10 120 python -u tools/probe/gemm_k_sweep.py > $OUT/ksweep_B.log 2>&1 || exit 1
tail -2 $OUT/ksweep_A.log $OUT/ksweep_B.log
A_ENV="" B_ENV="ARCWELD_LIB=$LX" timeout -k 10 900 bash tools/ab_lib.sh || exit 1
cp -r gpurun_out/ab_lib $OUT/ 2>/dev/null
echo done
