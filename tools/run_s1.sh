set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_s2
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "wgrad_batch or bf16_residual" > gpurun_out/r04_s2/k.log 2>&1 || { tail -40 gpurun_out/r04_s2/k.log; exit 1; }
tail -2 gpurun_out/r04_s2/k.log
TAG=r04_s2 STAGES="tests smoke" bash tools/evidence.sh || exit 1
VAR=ARCWELD_RESID_F32 bash tools/ab_env_bench.sh 1 0 2 || exit 1
VAR=ARCWELD_WGRAD_BATCH bash tools/ab_env_bench.sh 0 1 2 || exit 1
ARGS="--only transformer_pretokenized" VAR=ARCWELD_WGRAD_BATCH bash tools/ab_env_bench.sh 0 1 2 || exit 1
TAG=r04_s2 STAGES="bench" bash tools/evidence.sh
