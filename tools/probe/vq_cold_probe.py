"""The VQ forward (step form) with warm caches (back-to-back launches) and with cold ones (a 1 GiB copy between
launches evicts L2 and the MALL; the copy is outside the timed events): what the in-step launch pays for its codebook
and z coming from HBM.  Variant "touch": a one-workgroup-per-XCD read of the codebook just before each cold launch.
usage: python3 tools/probe/vq_cold_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd")]

import torch  # noqa: E402

from arcweld import kernels as K  # noqa: E402
from arcweld.vqvae import VQ_COUNT_GROUPS  # noqa: E402

N, Kc, D = 16384, 512, 64
g = torch.Generator(device="cuda").manual_seed(0)
z = torch.randn(N, D, device="cuda", generator=g) * 0.08
E = torch.randn(Kc, D, device="cuda", generator=g) * 0.08
zq = torch.empty_like(z)
zq2 = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
idx = torch.empty(N, dtype=torch.int64, device="cuda")
counts = torch.zeros(VQ_COUNT_GROUPS * Kc, device="cuda")
sq = torch.zeros(1, device="cuda", dtype=torch.float64)
big = [torch.empty(1 << 28, device="cuda"), torch.empty(1 << 28, device="cuda")]


def vq():
    K.vq_forward(z, E, zq, idx, counts, sq, zq_copy=zq2, count_groups=VQ_COUNT_GROUPS)


def timed(pre, n=20):
    ts = []
    for _ in range(n):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        vq()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for _ in range(3):
    vq()
print(f"warm (previous launch just ran): {timed(lambda: vq()):.1f} us")
print(f"cold (1 GiB copy between):       {timed(lambda: big[1].copy_(big[0])):.1f} us")


def cold_then_z():
    big[1].copy_(big[0])
    z.mul_(1.0)        # z rewritten just before, as the Ws GEMM writes it in the step


print(f"cold codebook, z just written:    {timed(cold_then_z):.1f} us")


def cold_then_both():
    big[1].copy_(big[0])
    z.mul_(1.0)
    E.mul_(1.0)


print(f"codebook and z just written:      {timed(cold_then_both):.1f} us")
