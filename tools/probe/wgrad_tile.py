"""Decoder weight-gradient grouped launch (16 x 512 x 1536 x 16384, implicit conv on B, accumulate) at the
128x128 and 256x128 tiles.  usage: python tools/probe/wgrad_tile.py"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import _native, kernels as K  # noqa: E402

H, S, G, M = 512, 16, 16, 16384
g = torch.Generator(device="cuda").manual_seed(0)
go = [torch.randn(M, H, device="cuda", generator=g).bfloat16() for _ in range(G)]
acts = [torch.randn(M, H, device="cuda", generator=g).bfloat16() for _ in range(G)]
gw = [torch.zeros(H, 3 * H, device="cuda") for _ in range(G)]
rs = [torch.zeros(H, device="cuda") for _ in range(G)]
probs = [(go[i], acts[i], H, 3 * H, M, dict(a_trans=True, b_trans=True, conv=(H, S, 1, 1), C=gw[i],
                                             accumulate=True, col_map=(H, 3, 0), a_rowsum=rs[i])) for i in range(G)]
for tile in (0, 256, 0, 256):
    _native.call("aw_gemm_set_tile", tile)
    for _ in range(3):
        K.gemm_grouped(probs)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        K.gemm_grouped(probs)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 10 * 1e3
    fl = G * 2 * H * 3 * H * M * (3 - 2 / S) / 3
    print(f"tile {tile or 128}: {us:7.1f} us  {fl / us / 1e6:6.1f} TF", flush=True)
