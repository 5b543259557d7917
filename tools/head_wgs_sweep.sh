set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/hw
for n in 128 256 512 1024; do
  AW_HEAD_WGS=$n timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hw/w$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-profile --no-transformer --steps 10 > gpurun_out/hw/w$n.json 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/hw/w$n/run_kernel_stats.csv')):
    n=r['Name']
    if any(k in n for k in ('head_','radam','sumsq')): print($n, n[:40], r['AverageNs'])
"
done
