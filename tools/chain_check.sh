#!/bin/bash
# Chain check on one GPU box: the chain tests, the chain probes (product library and the variants), and a
# same-box A/B of the VQ-VAE step against ./ab_base.  Stops at the first GPU fault / timeout (rc not in {0, 1}).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_pair}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_res_chain.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -25 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
for taps in 1 3; do
  timeout -k 10 120 python -u tools/probe/res_chain_probe.py 20 $taps > $OUT/probe_$taps.log 2>&1 || { cat $OUT/probe_$taps.log; exit 1; }
  cat $OUT/probe_$taps.log
done
for taps in 1 3; do
  timeout -k 10 200 python -u tools/probe/res_chain_variants.py 20 $taps > $OUT/var_$taps.log 2>&1 || { cat $OUT/var_$taps.log; exit 1; }
  cat $OUT/var_$taps.log
done
if [ -n "$AB" ]; then timeout -k 10 700 bash tools/ab_tree.sh || exit 1; fi
echo done
