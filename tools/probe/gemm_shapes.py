"""Per-call shapes and HIP-event durations of the plain aw_gemm launches of the configs[1] VQ-VAE step (eager, bf16):
which of the step's ~11 non-chain GEMMs cost what.  usage: python3 tools/probe/gemm_shapes.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from arcweld import kernels as K  # noqa: E402

orig = K.gemm
rows = []


def gemm(A, B, M, N, Kd, **kw):
    out = orig(A, B, M, N, Kd, **kw)
    if K.PROFILE is not None and K.PROFILE:
        e = K.PROFILE[-1]
        flags = [k for k in ("conv", "bias", "pre", "resid", "C2", "colstats", "a_rowsum", "accumulate", "drop")
                 if not (kw.get(k) is None or kw.get(k) is False or (isinstance(kw.get(k), tuple) and
                                                                      kw.get(k)[:1] == (0.0,)))]
        rows.append((M, N, Kd, int(kw.get("a_trans", False)), int(kw.get("b_trans", False)), ",".join(flags), e))
    return out


K.gemm = gemm      # the step's modules call K.gemm through the module attribute
dev = torch.device("cuda")


class A:
    batch, no_graph = 1024, True


bench.vqvae_workload(dev, 0, 1, A, torch.bfloat16, 3, 2, profile=True)
torch.cuda.synchronize()
n_prof = 3
agg = {}
for M, N, Kd, at, bt, fl, e in rows:
    k = (M, N, Kd, at, bt, fl)
    agg.setdefault(k, []).append(e[0].elapsed_time(e[1]) * 1e3)
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    M, N, Kd, at, bt, fl = k
    us = sum(v) / len(v)
    tot += sum(v) / n_prof
    tf = 2.0 * M * N * Kd / (us * 1e-6) / 1e12
    print(f"M {M:6d} N {N:5d} K {Kd:6d} aT {at} bT {bt} {fl:32s} x{len(v) // n_prof}  {us:7.1f} us  {tf:6.1f} TF/s")
print(f"total {tot:.1f} us per step")
