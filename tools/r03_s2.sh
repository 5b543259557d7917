set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_s2
mkdir -p $OUT
timeout -k 10 120 python -u tools/probe/wgrad3_probe.py 10 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad_conv3 or unpatch_head" -m gpu > $OUT/pytest_k.log 2>&1 || { tail -30 $OUT/pytest_k.log; exit 1; }
tail -2 $OUT/pytest_k.log
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python3 tools/probe/wgrad3_probe.py 3 > $OUT/pmc_sq.log 2>&1 || { tail -20 $OUT/pmc_sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-transformer --no-profile --steps 10 --warmup 3 > $OUT/vq_bench.log 2>&1 || { tail -30 $OUT/vq_bench.log; exit 1; }
grep -o '"value[^,]*,[^,]*,[^,]*,[^,]*,[^,]*,[^,]*' $OUT/vq_bench.log | head -2
echo done
