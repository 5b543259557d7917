#!/bin/bash
# Full evidence pass on one GPU box: gpu tests, the default bench line (roofline + cpu_baseline), the rocprofv3
# kernel-trace summary of the bench, and the two PMC passes for the GEMM family's HBM traffic.
# usage: TAG=name bash tools/gpu_round_full.sh   (outputs under gpurun_out/$TAG)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > $OUT/bench_under_rocprof.log 2>&1 || { tail -30 $OUT/bench_under_rocprof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transformer --no-profile --steps 5 --warmup 2 > $OUT/pmc_fetch.log 2>&1 || { tail -30 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-transformer --no-profile --steps 5 --warmup 2 > $OUT/pmc_write.log 2>&1 || { tail -30 $OUT/pmc_write.log; exit 1; }
echo done
