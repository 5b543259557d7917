set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_s11
mkdir -p $O
timeout -k 10 120 python -u tools/debug/bf16_small.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > $O/attn.log 2>&1 || { tail -30 $O/attn.log; exit 1; }
tail -1 $O/attn.log
for i in 1 2; do timeout -k 10 120 python tools/probe/attn_probe.py 50 2>&1 | grep -v amdgpu.ids | tr '\n' ' '; echo; done
timeout -k 10 300 python -u bench.py --only transformer_pretokenized --no-profile --detail "" 2>&1 | tail -1 | cut -c1-200
