# SQ counters of the VQ-VAE step's non-GEMM kernels (head, VQ, optimizer): instruction mix and waits
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmch
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM -d gpurun_out/pmch/a -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transformer --no-profile --steps 3 --warmup 2 > gpurun_out/pmch/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU -d gpurun_out/pmch/b -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transformer --no-profile --steps 3 --warmup 2 > gpurun_out/pmch/b.log 2>&1 || exit 1
