"""Attention kernels at the transformer bench shape (51 sequences x 321 tokens, 8 heads of 64): time per call of
the forward and the backward (delta + dQ + dK/dV), for rocprofv3 counter passes.
usage: python tools/probe/attn_probe.py [iters]"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import kernels as K  # noqa: E402

B, T, nh, d = 51, 321, 8, 512


def main(iters=20):
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * T, 3 * d, device="cuda", generator=g).bfloat16()
    y = torch.empty(B * T, d, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(B * T, d, device="cuda", generator=g).bfloat16()
    lse = torch.empty(B * nh * T, device="cuda")
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(B * nh * T, device="cuda")
    for name, fn in (("fwd", lambda: K.attn_fwd(qkv, B, T, nh, d, y, lse)),
                     ("bwd", lambda: K.attn_bwd(qkv, y, dy, lse, B, T, nh, d, dqkv, ws))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(iters):
            fn()
        t1.record()
        torch.cuda.synchronize()
        print(f"{name}: {t0.elapsed_time(t1) / iters * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
