"""Decoder conv input-gradient GEMMs (M 16384 tokens, N 512, K 3 x 512, implicit k = 3 conv with dir -1) with the
weight operand as today ([3O][I], read transposed: the 128-row tile) against a K-contiguous [I][3O] copy (eligible
for the 256-row ping-pong tile), both epilogue forms of the ResBlock backward (vqvae.py backward).
usage: python tools/probe/dgrad_tile_probe.py [iters]"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import kernels as K  # noqa: E402

N, H, S = 16384, 512, 16
bf = torch.bfloat16


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / iters * 1e3


def main(iters=50):
    g = torch.Generator(device="cuda").manual_seed(0)
    go = (torch.randn(N, H, device="cuda", generator=g) * 0.1).to(bf)
    Wt = (torch.randn(3 * H, H, device="cuda", generator=g) * 0.05).to(bf)     # [3O][I]
    Wk = Wt.t().contiguous()                                                   # [I][3O]
    pre = torch.randn(N, H, device="cuda", generator=g).to(bf)
    pref = torch.randn(N, H, device="cuda", generator=g)
    resid = torch.randn(N, H, device="cuda", generator=g)
    gh, ghk = torch.empty(N, H, device="cuda", dtype=bf), torch.empty(N, H, device="cuda", dtype=bf)
    gy, gyk = torch.empty(N, H, device="cuda"), torch.empty(N, H, device="cuda")
    g2, g2k = torch.empty(N, H, device="cuda", dtype=bf), torch.empty(N, H, device="cuda", dtype=bf)
    conv = (H, S, -1, 0)
    seed = torch.zeros(1, device="cuda", dtype=torch.int64)
    cases = {
        "conv2 dgrad [3O][I] b_trans": lambda: K.gemm(go, Wt, N, H, 3 * H, b_trans=True, conv=conv, pre=pre, C=gh),
        "conv2 dgrad [I][3O]": lambda: K.gemm(go, Wk, N, H, 3 * H, conv=conv, pre=pre, C=ghk),
        "conv1 dgrad [3O][I] b_trans": lambda: K.gemm(gh, Wt, N, H, 3 * H, b_trans=True, conv=conv, pre=pref,
                                                     resid=resid, C=gy, C2=g2, c2_mode=3, drop2=(0.1, 7),
                                                     seed_ptr=seed),
        "conv1 dgrad [I][3O]": lambda: K.gemm(gh, Wk, N, H, 3 * H, conv=conv, pre=pref, resid=resid, C=gyk, C2=g2k,
                                             c2_mode=3, drop2=(0.1, 7), seed_ptr=seed),
    }
    for name, fn in cases.items():
        print(f"{name}: {timeit(fn, iters):.1f} us", flush=True)
    torch.cuda.synchronize()
    for a, b in ((gh, ghk), (gy, gyk), (g2, g2k)):
        err = (a.float() - b.float()).abs().max().item()
        print("max |diff| between the two layouts:", err, flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
