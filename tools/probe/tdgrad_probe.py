"""The decoder's input-gradient GEMMs (model/transformer_block.py:28-30,76-77 backward: dX = dY . W with W in the
nn.Linear [out][in] layout, read transposed) against the same products with a K-contiguous copy W^T ([in][out]),
on the automatic tile and on forced 128- / 256-row tiles.  M = 51 x 321 tokens, bf16 operands, f32 output.
usage: python tools/probe/tdgrad_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
import torch  # noqa: E402

from arcweld import _native as nat  # noqa: E402
from arcweld import kernels as K  # noqa: E402


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    M = 51 * 321
    g = torch.Generator(device="cuda").manual_seed(0)
    for Kd, N in ((1536, 512), (2048, 512), (512, 2048), (512, 512)):
        dy = torch.randn(M, Kd, device="cuda", generator=g).bfloat16()
        W = torch.randn(Kd, N, device="cuda", generator=g).bfloat16()        # [out][in]: B read transposed
        Wt = W.t().contiguous()                                             # [in][out]: K-contiguous
        C = torch.empty(M, N, device="cuda")
        ref = dy.float() @ W.float()
        res = {}
        for tile in (0, 128, 256):
            nat.call("aw_gemm_set_tile", tile)
            res[f"trans t{tile}"] = timeit(lambda: K.gemm(dy, W, M, N, Kd, b_trans=True, C=C))
            err_t = float((C - ref).abs().max())
            res[f"kcontig t{tile}"] = timeit(lambda: K.gemm(dy, Wt, M, N, Kd, C=C))
            err_k = float((C - ref).abs().max())
            assert err_t < 1e-1 * ref.abs().max() and err_k < 1e-1 * ref.abs().max(), (err_t, err_k)
        nat.call("aw_gemm_set_tile", 0)
        fl = 2 * M * N * Kd
        print(f"K={Kd} N={N}: " + ", ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f} TF/s)" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
