set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_s4
mkdir -p $OUT
timeout -k 10 120 python -u tools/probe/wgrad3_probe.py 10 > $OUT/probe.log 2>&1 || { cat $OUT/probe.log; exit 1; }
cat $OUT/probe.log
