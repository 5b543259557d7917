set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_s2; mkdir -p $O
timeout -k 10 120 python -u tools/probe/enc_chain_probe.py 2>&1 | grep -v amdgpu.ids
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python -u $GRAFT_REPO_ROOT/tools/probe/enc_chain_probe.py 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
python $GRAFT_REPO_ROOT/tools/probe/kstats.py $GRAFT_REPO_ROOT/$O/prof | head -20
