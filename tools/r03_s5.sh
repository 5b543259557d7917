# GEMM 256-row ping-pong: kernel tests, VQ-VAE parity, same-box A/B of the step (auto policy vs 128-row tiles)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03_s5}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_vqvae_full_batch.py tests/test_vqvae_module.py -m gpu > $OUT/pytest_k.log 2>&1 || { tail -40 $OUT/pytest_k.log; exit 1; }
tail -2 $OUT/pytest_k.log
B="python3 bench.py --no-transformer --no-stress --no-fp32 --no-cpu-baseline --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 120 $B > $OUT/auto_$r.json 2>$OUT/auto_$r.err || { tail -5 $OUT/auto_$r.err; exit 1; }
  timeout -k 10 120 $B --gemm-tile 128 > $OUT/t128_$r.json 2>$OUT/t128_$r.err || { tail -5 $OUT/t128_$r.err; exit 1; }
  echo "run $r auto $(grep -o '"ms_per_step[^,]*' $OUT/auto_$r.json | head -1) t128 $(grep -o '"ms_per_step[^,]*' $OUT/t128_$r.json | head -1)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/vq -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-transformer --no-profile --steps 10 --warmup 3 > $OUT/vq_bench.log 2>&1 || { tail -30 $OUT/vq_bench.log; exit 1; }
echo done
