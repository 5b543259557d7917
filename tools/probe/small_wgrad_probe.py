"""The VQ-VAE step's three small weight gradients (patch embed 512 x 25, sep 64 x 512, dec0 512 x 64, K = 16384
tokens, accumulate + bias row sums) as the step issues them, HIP-event time per call (split-K plan of csrc/gemm.hip;
AW_SPLIT_MIN_KSTEPS_SMALL varies the fewest K steps per split).  usage: python3 tools/probe/small_wgrad_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "vq-vae-transformer-arc-welding_amd"))
from arcweld import kernels as K  # noqa: E402

dev = "cuda"
BF = torch.bfloat16
N = 16384
g = torch.Generator(device=dev).manual_seed(0)
cases = {
    "patch 512x25": (torch.randn(N, 512, device=dev, generator=g).to(BF), torch.randn(N, 32, device=dev, generator=g).to(BF), 512, 25),
    "sep 64x512": (torch.randn(N, 64, device=dev, generator=g).to(BF), torch.randn(N, 512, device=dev, generator=g).to(BF), 64, 512),
    "dec0 512x64": (torch.randn(N, 512, device=dev, generator=g).to(BF), torch.randn(N, 64, device=dev, generator=g).to(BF), 512, 64),
}
res = {}
for name, (A, B, M, Nn) in cases.items():
    C = torch.zeros(M, Nn, device=dev)
    rs = torch.zeros(M, device=dev)
    ref = (A.float().t() @ B.float()[:, :Nn])

    def run():
        K.gemm(A, B, M, Nn, N, a_trans=True, b_trans=True, C=C, accumulate=True, a_rowsum=rs)
    for _ in range(5):
        run()
    C.zero_()
    rs.zero_()
    run()
    torch.cuda.synchronize()
    err = float((C - ref).abs().max() / ref.abs().max())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    res[name] = (e0.elapsed_time(e1) * 1e3 / 50, err)
print(os.environ.get("AW_SPLIT_MIN_KSTEPS_SMALL", "default"),
      "  ".join(f"{k}: {v[0]:.1f} us (rel err {v[1]:.1e})" for k, v in res.items()))
