#!/bin/bash
# One GPU call: rocprofv3 kernel trace + stats of the configs[2] decoder train step alone (bench.py --only
# transformer_pretokenized), then the SQ / FETCH_SIZE / WRITE_SIZE PMC passes of the same command, each its own run
# (MI355X_MICROARCH.md).  usage: TAG=r03 bash tools/prof_transformer.sh  -> gpurun_out/proft_$TAG/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/proft_${TAG:-run}
mkdir -p $OUT
CMD="python3 bench.py --only transformer_pretokenized --no-profile --steps ${STEPS:-10} --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- $CMD > $OUT/pmc_sq.log 2>&1 || { tail -20 $OUT/pmc_sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $CMD > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $CMD > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
# per-kernel HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE) -> the record bench.py's roofline reads once committed
# under profiles/r<round>/<session>/pmc_traffic_transformer.json, and the per-family summary (MFMA busy, LDS bank conflicts, GB/s)
python3 tools/pmc_traffic.py $(ls $OUT/pmc_fetch/*counter_collection.csv | head -1) $(ls $OUT/pmc_write/*counter_collection.csv | head -1) > $OUT/pmc_traffic_transformer.json || exit 1
python3 tools/pmc_summary.py $OUT $OUT/pmc_summary.json > /dev/null || exit 1
cp $(ls $OUT/trace/*kernel_stats.csv | head -1) $OUT/kernel_stats.csv
echo done
