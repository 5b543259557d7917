# PMC passes (SQ timing / MFMA / LDS; TA / L2 hits) over tools/probe/wgrad_probe.py: the grouped weight-gradient kernels
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_wgrad
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_wgrad/a -o run --output-format csv -- python3 tools/probe/wgrad_probe.py 3 > gpurun_out/pmc_wgrad/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS -d gpurun_out/pmc_wgrad/b -o run --output-format csv -- python3 tools/probe/wgrad_probe.py 3 > gpurun_out/pmc_wgrad/b.log 2>&1 || exit 1
echo ok
