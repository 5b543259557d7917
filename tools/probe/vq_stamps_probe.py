"""Phase stamps of the codebook-pinned VQ forward (a probe build of csrc/vq.hip with s_memtime stamps at its phase
boundaries, tools/probe/build/vqs.so, built by hand): median cycles per phase over the first 256 workgroups.
usage on the GPU box: python tools/probe/vq_stamps_probe.py [vqs_<variant>.so]"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAME = sys.argv[1] if len(sys.argv) > 1 else "vqs.so"
lib = ctypes.CDLL(os.path.join(HERE, "build", NAME))
N, Kc, D = 16384, 512, 64
g = torch.Generator(device="cuda").manual_seed(0)
z = torch.randn(N, D, device="cuda", generator=g) * 0.08
E = torch.randn(Kc, D, device="cuda", generator=g) * 0.08
zq = torch.empty_like(z)
idx = torch.empty(N, dtype=torch.int64, device="cuda")
counts = torch.zeros(Kc, device="cuda")
sq = torch.zeros(1, device="cuda", dtype=torch.float64)
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p
for _ in range(5):
    assert lib.aw_vq_forward(P(z.data_ptr()), P(E.data_ptr()), ctypes.c_int64(N), Kc, D, P(zq.data_ptr()),
                             P(idx.data_ptr()), P(counts.data_ptr()), P(sq.data_ptr()), P(s)) == 0
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(20):
    lib.aw_vq_forward(P(z.data_ptr()), P(E.data_ptr()), ctypes.c_int64(N), Kc, D, P(zq.data_ptr()),
                      P(idx.data_ptr()), P(counts.data_ptr()), P(sq.data_ptr()), P(s))
ev[1].record()
torch.cuda.synchronize()
print(f"{NAME}: {ev[0].elapsed_time(ev[1]) / 20 * 1e3:.1f} us per launch (events, 20 back to back)")
buf = (ctypes.c_uint64 * (256 * 8 * 16))()
lib.vq_probe_stamps(buf)
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, 16).astype(np.int64)
if (st[:, :, 6] == 0).any():
    sys.exit(0)   # a variant that leaves before the last stamp: launch time only
names = ["loads-issue+z", "chunks (mfma)", "norms publish", "argmin", "merge+barrier", "finish"]
t0 = st[:, :, 0].min(axis=1, keepdims=True)            # each workgroup's first wave start
rel = st[:, :, :7] - t0[:, :, None]                    # [wg][wave][stamp] cycles since the workgroup started
print("stamp times since the workgroup's start (cycles; median over WGs of the earliest / latest wave):")
for k in range(7):
    lo, hi = np.median(rel[:, :, k].min(axis=1)), np.median(rel[:, :, k].max(axis=1))
    print(f"  after {(['start'] + names)[k]:16s} earliest {int(lo):6d}  latest {int(hi):6d}")
rt = st[:, :, 9].max(axis=1) - st[:, :, 8].min(axis=1)   # 100 MHz ticks
clk = (st[:, :, 6].max(axis=1) - st[:, :, 0].min(axis=1)) / (rt / 100e6) / 1e9
print(f"shader clock from s_memtime / s_memrealtime: median {np.median(clk):.2f} GHz")
print(f"per-WG duration (real time): median {np.median(rt) * 10 / 1e3:.2f} us  max {rt.max() * 10 / 1e3:.2f} us")
print(f"first start -> last end {(st[:, :, 9].max() - st[:, :, 8].min()) * 10 / 1e3:.2f} us")
sys.stdout.flush()
