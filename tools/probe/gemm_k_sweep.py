"""Fixed cost vs per-K-step cost of the 128x128 GEMM: plain bf16 (C only) M 16384, N 512 over K, fitted as
T(K) = T0 + (K / 64) * t_step.  usage: python tools/probe/gemm_k_sweep.py"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import _native, kernels as K  # noqa: E402
import os  # noqa: E402

_native.call("aw_gemm_set_tile", int(os.environ.get("TILE", "0")))

M, N = 16384, 512


def t(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


ks, ts = [], []
for Kd in (256, 512, 1024, 1536, 3072, 6144):
    A = torch.randn(M, Kd, device="cuda").bfloat16()
    B = torch.randn(N, Kd, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Cf = torch.empty(M, N, device="cuda")
    us = t(lambda: K.gemm(A, B, M, N, Kd, C=C))
    usf = t(lambda: K.gemm(A, B, M, N, Kd, C=Cf))
    ks.append(Kd / 64)
    ts.append(us)
    print(f"K {Kd:5d}: bf16 C {us:7.1f} us  f32 C {usf:7.1f} us  ({2 * M * N * Kd / us / 1e6:6.1f} TF)", flush=True)
n = len(ks)
mx, my = sum(ks) / n, sum(ts) / n
slope = sum((x - mx) * (y - my) for x, y in zip(ks, ts)) / sum((x - mx) ** 2 for x in ks)
print(f"fit: T0 = {my - slope * mx:.1f} us, t_step = {slope:.3f} us per 64-deep K step "
      f"(MFMA-bound step at 2.5 PF: {2 * M * N * 64 / 2.5e15 * 1e6:.3f} us)")
