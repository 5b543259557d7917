"""LayerNorm backward at the transformer bench shape (51 x 321 rows of 512, accumulate into the residual gradient,
bf16 operand copy of dx): time per call.  AW_LN_BWD_BLOCKS sweeps the workgroup count.
usage: python tools/probe/ln_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd")]

import torch  # noqa: E402

from arcweld import kernels as K  # noqa: E402


def main(iters=30):
    R, D = 51 * 321, 512
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(R, D, device="cuda", generator=g)
    dy = torch.randn(R, D, device="cuda", generator=g)
    w, b = torch.randn(D, device="cuda", generator=g), torch.randn(D, device="cuda", generator=g)
    y, mean, rstd = torch.empty(R, D, device="cuda", dtype=torch.bfloat16), torch.empty(R, device="cuda"), \
        torch.empty(R, device="cuda")
    K.layernorm_fwd(x, w, b, 1e-5, y, mean, rstd)
    dx, dw, db = torch.zeros(R, D, device="cuda"), torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    dx2 = torch.empty(R, D, device="cuda", dtype=torch.bfloat16)
    for name, fn in (("fwd", lambda: K.layernorm_fwd(x, w, b, 1e-5, y, mean, rstd)),
                     ("bwd", lambda: K.layernorm_bwd(x, dy, w, mean, rstd, dx, True, dw, db, dx2=dx2))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(iters):
            fn()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) / iters * 1e3
        nbytes = R * D * (4 + 2) if name == "fwd" else R * D * (4 + 4 + 4 + 4 + 2)
        print(f"{name} blocks={os.environ.get('AW_LN_BWD_BLOCKS', 512)}: {us:.1f} us  {nbytes / us / 1e3:.0f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
