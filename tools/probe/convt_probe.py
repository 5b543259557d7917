"""The un-patch ConvT forward GEMM of the configs[1] step (M 16384 x N 2560 x K 512, bf16, bias per channel, the
BatchNorm column statistics folded to 512 channels by f64 atomics) with and without the statistics epilogue, HIP
events over 50 calls.  usage: python3 tools/probe/convt_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "vq-vae-transformer-arc-welding_amd"))
from arcweld import kernels as K  # noqa: E402

BF = torch.bfloat16
N, H, k1 = 16384, 512, 5
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(N, H, device="cuda", generator=g).to(BF)
W = (torch.randn(k1 * H, H, device="cuda", generator=g) * 0.04).to(BF)
b = torch.randn(H, device="cuda", generator=g)
Y = torch.empty(N, k1 * H, device="cuda", dtype=BF)
cs = torch.zeros(2 * H, device="cuda", dtype=torch.float64)


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


t1 = timeit(lambda: K.gemm(A, W, N, k1 * H, H, bias=b, bias_mod=H, C=Y, colstats=cs, stats_mod=H))
t0 = timeit(lambda: K.gemm(A, W, N, k1 * H, H, bias=b, bias_mod=H, C=Y))
print(f"ConvT forward GEMM: with column statistics {t1:.1f} us, without {t0:.1f} us")
