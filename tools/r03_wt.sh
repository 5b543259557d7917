#!/bin/bash
# A/B: write-through (sc1) GEMM epilogue stores vs non-temporal, class-A launches and the bench step.
set -o pipefail
mkdir -p gpurun_out/wt
timeout -k 10 120 python -u tools/probe/classa_waves.py > gpurun_out/wt/waves_nt.log 2>&1 || exit 1
ARCWELD_LIB=tools/probe/build/libarcweld_wt.so timeout -k 10 120 python -u tools/probe/classa_waves.py > gpurun_out/wt/waves_wt.log 2>&1 || exit 1
bash tools/ab_bench.sh vq-vae-transformer-arc-welding_amd/lib/libarcweld_amd.so tools/probe/build/libarcweld_wt.so 2 > gpurun_out/wt/ab.log 2>&1
