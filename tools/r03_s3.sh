set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_s3
mkdir -p $OUT
timeout -k 10 120 python -u tools/probe/wgrad3_probe.py 10 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python3 tools/probe/wgrad3_probe.py 2 > $OUT/pmc_sq.log 2>&1 || { tail -20 $OUT/pmc_sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 tools/probe/wgrad3_probe.py 2 > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
echo done
