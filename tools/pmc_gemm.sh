# SQ counter passes over the plain bf16 GEMM probe (16384 x 512 x 1536): where the main loop's time goes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcg
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS -d gpurun_out/pmcg/a -o run --output-format csv -- python3 tools/probe/stream_split.py plain_bf16 > gpurun_out/pmcg/a.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM -d gpurun_out/pmcg/b -o run --output-format csv -- python3 tools/probe/stream_split.py plain_bf16 > gpurun_out/pmcg/b.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmcg/c -o run --output-format csv -- python3 tools/probe/stream_split.py plain_bf16 > gpurun_out/pmcg/c.log 2>&1 || exit 1
