"""Phase stamps of the codebook-pinned VQ forward (a probe build of csrc/vq.hip with s_memtime stamps at its phase
boundaries, tools/probe/build/vqs.so, built by hand): median cycles per phase over the first 256 workgroups.
usage on the GPU box: python tools/probe/vq_stamps_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "build", "vqs.so"))
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
buf = (ctypes.c_uint64 * (256 * 8))()
lib.vq_probe_stamps(buf)
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8).astype(np.int64)[:, :6]
d = np.diff(st, axis=1)
print("phase cycles (median over WGs): loads+transpose %d  norms %d  main loop %d  argmin %d  finish %d  total %d" %
      tuple(list(np.median(d, axis=0).astype(int)) + [int(np.median(st[:, 5] - st[:, 0]))]))
print("start spread (cycles):", int(st[:, 0].max() - st[:, 0].min()), " end spread:", int(st[:, 5].max() - st[:, 5].min()))
sys.stdout.flush()
