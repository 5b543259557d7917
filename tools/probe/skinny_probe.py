"""Isolated timings of the VQ-VAE step's un-patch ConvT forward and its three skinny weight gradients (decoder 1x1
conv, SepCNN conv, patch embed: M x N <= 512 x 64 over K = 16384 tokens, split over K with a slab reduce).

usage: python tools/probe/skinny_probe.py [iters]     (ARCWELD_LIB selects the library build)
ConvT variants: as in the step (bias, BN column statistics, bf16 Y), without the statistics, without bias and
statistics, and on the forced 256-row tile (checked equal to the 128-row output first)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
import torch  # noqa: E402

from arcweld import _native as nat  # noqa: E402
from arcweld import kernels as K  # noqa: E402

dev = "cuda"
bf = torch.bfloat16
IT = int(sys.argv[1]) if len(sys.argv) > 1 else 30


def timeit(fn, n=IT):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    torch.manual_seed(0)
    N, H, D, k1 = 16384, 512, 64, 5
    out = []
    # ---- ConvT forward (vqvae.py forward: K.gemm(yR_T, Wt1, N, k1*H, H, bias, bias_mod=H, C=Y, colstats))
    A = torch.randn(N, H, device=dev).to(bf)
    W = (torch.randn(k1 * H, H, device=dev) * 0.05).to(bf)
    bias = torch.randn(H, device=dev)
    Y = torch.empty(N, k1 * H, device=dev, dtype=bf)
    cs = torch.zeros(2 * H, device=dev, dtype=torch.float64)
    step = lambda: K.gemm(A, W, N, k1 * H, H, bias=bias, bias_mod=H, C=Y, colstats=cs, stats_mod=H)  # noqa: E731
    out.append(("convt fwd (step form)", timeit(step)))
    out.append(("convt fwd no colstats", timeit(lambda: K.gemm(A, W, N, k1 * H, H, bias=bias, bias_mod=H, C=Y))))
    out.append(("convt fwd plain", timeit(lambda: K.gemm(A, W, N, k1 * H, H, C=Y))))
    cs.zero_()
    step()
    ref_y, ref_cs = Y.clone(), cs.clone()
    nat.load().aw_gemm_set_tile(256)
    try:
        cs.zero_()
        step()
        torch.cuda.synchronize()
        dy = (Y.float() - ref_y.float()).abs().max().item()
        dcs = ((cs - ref_cs).abs().max() / ref_cs.abs().max()).item()
        out.append((f"convt fwd tile256 (dY {dy:.2e}, dstats {dcs:.1e})", timeit(step)))
    finally:
        nat.load().aw_gemm_set_tile(0)
    # ---- skinny weight gradients (vqvae.py backward)
    go = torch.randn(N, H, device=dev).to(bf)
    zq = torch.randn(N, D, device=dev).to(bf)
    pt = torch.randn(N, 32, device=dev).to(bf)
    Cd, rb = torch.zeros(H, D, device=dev), torch.zeros(H, device=dev)
    Cs, rs = torch.zeros(D, H, device=dev), torch.zeros(D, device=dev)
    Cp = torch.zeros(H, 25, device=dev)
    kw = dict(a_trans=True, b_trans=True, accumulate=True)
    out.append(("wgrad dec0 512x64", timeit(lambda: K.gemm(go, zq, H, D, N, C=Cd, a_rowsum=rb, **kw))))
    out.append(("wgrad sep 64x512", timeit(lambda: K.gemm(zq, go, D, H, N, C=Cs, a_rowsum=rs, **kw))))
    out.append(("wgrad pe 512x25", timeit(lambda: K.gemm(go, pt, H, 25, N, C=Cp, a_rowsum=rb, **kw))))
    # correctness of the split path against torch (fp32 of the same bf16 operands)
    Cd.zero_(), rb.zero_()
    K.gemm(go, zq, H, D, N, C=Cd, a_rowsum=rb, **kw)
    ref = go.float().t() @ zq.float()
    err = ((Cd - ref).abs().max() / ref.abs().max()).item()
    for name, us in out:
        print(f"{name:48s} {us:8.2f} us")
    print(f"dec0 wgrad rel err {err:.2e}")


if __name__ == "__main__":
    main()
