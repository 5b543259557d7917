# epilogue-operand prefetch: kernel tests, then same-box A/B of the step (prefetch on / off)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_s6}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_vqvae_full_batch.py -m gpu > $OUT/pytest_k.log 2>&1 || { tail -40 $OUT/pytest_k.log; exit 1; }
tail -2 $OUT/pytest_k.log
B="python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 120 $B > $OUT/pf_$r.json 2>$OUT/pf_$r.err || { tail -5 $OUT/pf_$r.err; exit 1; }
  ARCWELD_GEMM_PF=0 timeout -k 10 120 $B > $OUT/nopf_$r.json 2>$OUT/nopf_$r.err || { tail -5 $OUT/nopf_$r.err; exit 1; }
  echo "run $r pf $(grep -o '"ms_per_step[^,]*' $OUT/pf_$r.json | head -1) nopf $(grep -o '"ms_per_step[^,]*' $OUT/nopf_$r.json | head -1)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-transformer --no-profile --steps 10 --warmup 3 > $OUT/vq_bench.log 2>&1 || { tail -30 $OUT/vq_bench.log; exit 1; }
ARCWELD_GEMM_PF=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vq0 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-transformer --no-profile --steps 10 --warmup 3 > $OUT/vq0_bench.log 2>&1 || { tail -30 $OUT/vq0_bench.log; exit 1; }
echo done
