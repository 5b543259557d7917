"""The decoder's mlp.c_fc forward GEMM (M 16371 x N 2048 x K 512, bf16, bias, C = h and C2 = GELU_tanh(h)) and its
backward twin (gh = (go Wp) * GELU_tanh'(h)): where their time goes -- as the step calls them, with a single output,
without the activation, on the 256-row tile.  HIP events over 50 calls.  usage: python3 tools/probe/fc_gemm_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "vq-vae-transformer-arc-welding_amd"))
from arcweld import _native as nat  # noqa: E402
from arcweld import kernels as K  # noqa: E402

BF = torch.bfloat16
R, d = 16371, 512
g = torch.Generator(device="cuda").manual_seed(0)
a2 = torch.randn(R, d, device="cuda", generator=g).to(BF)
Wfc = (torch.randn(4 * d, d, device="cuda", generator=g) * 0.04).to(BF)
bfc = torch.randn(4 * d, device="cuda", generator=g) * 0.1
h, gg = torch.empty(R, 4 * d, device="cuda", dtype=BF), torch.empty(R, 4 * d, device="cuda", dtype=BF)
go = torch.randn(R, d, device="cuda", generator=g).to(BF)
Wp = (torch.randn(d, 4 * d, device="cuda", generator=g) * 0.02).to(BF)
gh = torch.empty(R, 4 * d, device="cuda", dtype=BF)


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


fl = 2.0 * R * 4 * d * d
cases = {
    "fc fwd as in the step (h + GELU_tanh(h))": lambda: K.gemm(a2, Wfc, R, 4 * d, d, bias=bfc, act=K.AW_ACT_GELU_TANH,
                                                                C=h, C2=gg, c2_mode=1),
    "fc fwd, h only": lambda: K.gemm(a2, Wfc, R, 4 * d, d, bias=bfc, C=h),
    "fc fwd, no bias, h only": lambda: K.gemm(a2, Wfc, R, 4 * d, d, C=h),
    "gh bwd as in the step (act' of h)": lambda: K.gemm(go, Wp, R, 4 * d, d, b_trans=True, act=K.AW_ACT_GELU_TANH,
                                                         pre=h, C=gh),
    "gh bwd, no act'": lambda: K.gemm(go, Wp, R, 4 * d, d, b_trans=True, C=gh),
    "fc fwd, C = GELU(h), C2 = GELU'(h) (mode 4)": lambda: K.gemm(a2, Wfc, R, 4 * d, d, bias=bfc,
                                                                   act=K.AW_ACT_GELU_TANH, C=gg, C2=h, c2_mode=4),
    "gh bwd times the saved GELU'": lambda: K.gemm(go, Wp, R, 4 * d, d, b_trans=True, act=K.AW_ACT_DERIV, pre=h,
                                                   C=gh),
}
for tile in (0,):
    nat.load().aw_gemm_set_tile(tile)
    for name, fn in cases.items():
        us = timeit(fn)
        print(f"tile {tile or 'auto':>4}  {name:44s} {us:7.1f} us  {fl / us / 1e6:6.0f} TF/s", flush=True)
nat.load().aw_gemm_set_tile(0)
