"""VQ forward kernel timing (aw_vq_forward) at the configs[1] shape (N 16384, K 512 x D 64) and the stress shape
(N 16384, K 8192 x D 256): HIP-event time per launch, FP32 TFLOP/s (2*N*K*D) and the fraction of the 157.3 TF
fp32 peak.  usage: python tools/probe/vq_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd")]

import torch  # noqa: E402

from arcweld import kernels as K  # noqa: E402


def run(N, Kc, D, iters=20, step_form=False):
    """step_form: called as arcweld/vqvae.py calls it (bf16 operand copy of z_q, VQ_COUNT_GROUPS partial counts)."""
    from arcweld.vqvae import VQ_COUNT_GROUPS
    cg = VQ_COUNT_GROUPS if step_form else 1
    g = torch.Generator(device="cuda").manual_seed(0)
    z = torch.randn(N, D, device="cuda", generator=g) * 0.08
    E = torch.randn(Kc, D, device="cuda", generator=g) * 0.08
    zq = torch.empty_like(z)
    zq2 = torch.empty(N, D, device="cuda", dtype=torch.bfloat16) if step_form else None
    idx = torch.empty(N, dtype=torch.int64, device="cuda")
    counts = torch.zeros(cg * Kc, device="cuda")
    sq = torch.zeros(1, device="cuda", dtype=torch.float64)
    for _ in range(3):
        K.vq_forward(z, E, zq, idx, counts, sq, zq_copy=zq2, count_groups=cg)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        K.vq_forward(z, E, zq, idx, counts, sq, zq_copy=zq2, count_groups=cg)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    ref = torch.cdist(z, E).argmin(1)
    agree = (ref == idx).float().mean().item()
    tf = 2.0 * N * Kc * D / (us * 1e-6) / 1e12
    print(f"N {N} K {Kc} D {D}{' (step form)' if step_form else ''}: {us:8.1f} us  {tf:6.1f} TFLOP/s  "
          f"frac {tf / 157.3:.3f}  argmin agreement vs cdist {agree:.5f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "stress":
        run(16384, 8192, 256, iters=5)
    else:
        run(16384, 512, 64)
        run(16384, 512, 64, step_form=True)
        run(16384, 8192, 256)
        run(4096, 8192, 256)
