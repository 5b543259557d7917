set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmca
timeout -k 10 60 python tools/probe/attn_probe.py || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmca/a -o run --output-format csv -- python3 tools/probe/attn_probe.py 5 > gpurun_out/pmca/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM -d gpurun_out/pmca/b -o run --output-format csv -- python3 tools/probe/attn_probe.py 5 > gpurun_out/pmca/b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU -d gpurun_out/pmca/c -o run --output-format csv -- python3 tools/probe/attn_probe.py 5 > gpurun_out/pmca/c.log 2>&1 || exit 1
