set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s5
mkdir -p $O
timeout -k 10 300 python -u tools/debug/rccl_b2.py > $O/rccl_b2.log 2>&1; echo "rccl_b2 rc=$?"; grep -E "b2|Error" $O/rccl_b2.log | cut -c1-900
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > $O/attn.log 2>&1 || { tail -30 $O/attn.log; exit 1; }
tail -1 $O/attn.log
for v in 0 1 0 1; do ARCWELD_ATTN_FWD_HEAD=$v timeout -k 10 120 python tools/probe/attn_probe.py 50 > $O/attn_probe_$v.log 2>&1 || exit 1; echo "head=$v $(cat $O/attn_probe_$v.log | tr '\n' ' ')"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tv -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --no-stress --no-profile --no-transformer --steps 10 --warmup 3 --detail "" > $O/tv.log 2>&1 || { tail -20 $O/tv.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tt -o run --output-format csv -- python3 bench.py --only transformer_pretokenized --no-profile --steps 10 --warmup 3 --detail "" > $O/tt.log 2>&1 || { tail -20 $O/tt.log; exit 1; }
echo done
