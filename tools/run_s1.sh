set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s7
mkdir -p $O
for v in 0 1; do
ARCWELD_TAP3=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tv$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-profile --no-transformer --steps 10 --warmup 3 --detail "" > $O/tv$v.log 2>&1 || { tail -20 $O/tv$v.log; exit 1; }
done
echo done
