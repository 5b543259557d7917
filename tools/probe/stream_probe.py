"""Streaming-read calibration: torch reductions vs the grad-norm kernel over the same 67 MB (16.8M f32)."""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import kernels as K  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


n = 16_800_000
x = torch.randn(n, device="cuda")
y = torch.empty_like(x)
print(f"torch sum      {t(lambda: x.sum()):7.1f} us  ({n * 4 / t(lambda: x.sum()) / 1e3:.2f} TB/s)")
print(f"torch copy     {t(lambda: y.copy_(x)):7.1f} us")
off = torch.zeros(1, dtype=torch.int64, device="cuda")
ln = torch.full((1,), n, dtype=torch.int64, device="cuda")
act = torch.ones(1, dtype=torch.int32, device="cuda")
ws = torch.zeros(K.NORM_WS, dtype=torch.float64, device="cuda")
nm, cf = torch.zeros((), device="cuda"), torch.zeros((), device="cuda")
us = t(lambda: K.grad_norm_clip(x, off, ln, act, 1, 1.0, ws, nm, cf))
print(f"grad_norm_clip {us:7.1f} us  ({n * 4 / us / 1e3:.2f} TB/s)")
