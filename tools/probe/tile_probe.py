"""The decoder's forward GEMMs at the configs[2] shape (16371 rows, d 512) on the automatic tile and forced onto the
256-row ping-pong tile (aw_gemm_set_tile): c_attn (N 1536, bias, bf16 C), attn.c_proj and mlp.c_proj (N 512, bias +
dropout + residual, f32 C; K 512 / 2048), c_fc (N 2048, c_fc mode 4).  HIP events over 50 calls.
usage: python3 tools/probe/tile_probe.py"""
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
rn = lambda *s, dt=torch.float32, sc=1.0: (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)  # noqa: E731
ctr = torch.tensor([3], device="cuda", dtype=torch.int64)
a, y, gg = rn(R, d, dt=BF), rn(R, d, dt=BF), rn(R, 4 * d, dt=BF)
Wqkv, Wo, Wfc, Wp = rn(3 * d, d, dt=BF, sc=0.04), rn(d, d, dt=BF, sc=0.04), rn(4 * d, d, dt=BF, sc=0.04), \
    rn(d, 4 * d, dt=BF, sc=0.02)
b3, b1, b4 = rn(3 * d), rn(d), rn(4 * d)
qkv, x, x1 = torch.empty(R, 3 * d, device="cuda", dtype=BF), rn(R, d), torch.empty(R, d, device="cuda")
h, g2 = torch.empty(R, 4 * d, device="cuda", dtype=BF), torch.empty(R, 4 * d, device="cuda", dtype=BF)


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


cases = {
    "c_attn (N 1536, K 512)": lambda: K.gemm(a, Wqkv, R, 3 * d, d, bias=b3, C=qkv),
    "attn.c_proj (N 512, K 512)": lambda: K.gemm(y, Wo, R, d, d, bias=b1, drop=(0.1, 7), resid=x, C=x1, seed_ptr=ctr),
    "c_fc mode 4 (N 2048, K 512)": lambda: K.gemm(a, Wfc, R, 4 * d, d, bias=b4, act=K.AW_ACT_GELU_TANH, C=g2, C2=h,
                                                  c2_mode=4),
    "mlp.c_proj (N 512, K 2048)": lambda: K.gemm(gg, Wp, R, d, 4 * d, bias=b1, drop=(0.1, 8), resid=x, C=x1,
                                                 seed_ptr=ctr),
}
for name, fn in cases.items():
    res = []
    for tile in (0, 256, 128):
        nat.load().aw_gemm_set_tile(tile)
        res.append(timeit(fn))
    nat.load().aw_gemm_set_tile(0)
    print(f"{name:32s} auto {res[0]:6.1f}  256 {res[1]:6.1f}  128 {res[2]:6.1f} us", flush=True)
