set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_vq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_vq/a -o run --output-format csv -- python3 tools/probe/vq_probe.py stress > gpurun_out/pmc_vq/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VALU -d gpurun_out/pmc_vq/b -o run --output-format csv -- python3 tools/probe/vq_probe.py stress > gpurun_out/pmc_vq/b.log 2>&1 || exit 1
echo ok
