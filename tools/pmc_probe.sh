set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for v in bf16 plain_bf16; do
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA -d gpurun_out/pmc/$v -o run --output-format csv -- python3 tools/probe/stream_split.py $v > gpurun_out/pmc/$v.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS TA_BUSY_avr -d gpurun_out/pmc/${v}_2 -o run --output-format csv -- python3 tools/probe/stream_split.py $v > gpurun_out/pmc/${v}_2.log 2>&1 || exit 1
done
