"""Does splitting the batch into independent chains on separate streams overlap one chain's epilogue (HBM-bound)
with another's main loop (MFMA-bound)?  A chain of `depth` decoder-conv-like launches (M rows, N 512, K 1536
implicit conv, bias + dropout + residual epilogue, f32 C + bf16 C2) is captured in one HIP graph as 1, 2 or 4
independent chains of M/nchain rows each, fork/joined across streams.  usage: python tools/probe/stream_split.py"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import kernels as K  # noqa: E402

H, S, depth, M = 512, 16, 16, 16384


def chain_bufs(m):
    g = torch.Generator(device="cuda").manual_seed(0)
    y = [torch.randn(m, H, device="cuda", generator=g) for _ in range(2)]
    y += [torch.randn(m, 3 * H, device="cuda", generator=g).bfloat16() for _ in range(2)]
    a = [torch.randn(m, H, device="cuda", generator=g).bfloat16() for _ in range(2)]
    return y, a


EPI = "full"


def run_chain(y, a, W, bias, ctr, m):
    for i in range(depth):
        src, dst = i % 2, (i + 1) % 2
        if EPI == "full":
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, S, 1, 0), bias=bias, drop=(0.1, 1234 + i), seed_ptr=ctr,
                   resid=y[src], C=y[dst], C2=a[dst], c2_mode=1)
        elif EPI == "bf16":           # plain bf16 output
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, S, 1, 0), C=a[dst])
        elif EPI == "f32":
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, S, 1, 0), C=y[dst])
        elif EPI == "full_plain":     # same epilogue, dense K = 1536 operand (no implicit conv)
            K.gemm(y[src + 2], W, m, H, 3 * H, bias=bias, drop=(0.1, 1234 + i), seed_ptr=ctr,
                   resid=y[src], C=y[dst], C2=a[dst], c2_mode=1)
        elif EPI == "c1":             # conv1 form: bf16 pre-activation + bf16 GELU operand
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, S, 1, 0), bias=bias, C=a[dst], C2=a[src], c2_mode=1)
        elif EPI == "c1_plain":
            K.gemm(y[src + 2], W, m, H, 3 * H, bias=bias, C=a[dst], C2=a[src], c2_mode=1)
        elif EPI == "conv_noseg":     # implicit conv, one long segment (masks only at the ends)
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, m, 1, 0), C=a[dst])
        elif EPI == "conv_noshift":   # implicit conv with dir 0 (every tap reads the unshifted rows)
            K.gemm(a[src], W, m, H, 3 * H, conv=(H, S, 0, 0), C=a[dst])
        elif EPI == "plain_bf16":     # no implicit conv: dense K = 1536 operand
            K.gemm(y[src + 2], W, m, H, 3 * H, b_trans=False, C=a[dst])


def measure(nchain, iters=10):
    m = M // nchain
    W = (torch.randn(H, 3 * H, device="cuda") * 0.02).bfloat16()
    bias = torch.zeros(H, device="cuda")
    ctr = torch.zeros(1, device="cuda", dtype=torch.int64)
    bufs = [chain_bufs(m) for _ in range(nchain)]
    streams = [torch.cuda.Stream() for _ in range(nchain)]
    def body():
        main = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(main)
        for s in streams:
            s.wait_event(ev)
        for c, s in enumerate(streams):
            with torch.cuda.stream(s):
                run_chain(*bufs[c], W, bias, ctr, m)
        for s in streams:
            e = torch.cuda.Event()
            e.record(s)
            main.wait_event(e)

    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) / iters * 1e3
    print(f"chains {nchain}: {us:8.1f} us per {depth} launches = {us / depth:6.1f} us per full-M launch", flush=True)


if __name__ == "__main__":
    import os
    from arcweld import _native
    _native.call("aw_gemm_set_tile", int(os.environ.get("TILE", "0")))
    measure(1)          # clock warm-up
    if len(sys.argv) > 1:
        EPI = sys.argv[1]
        measure(1)
    else:
        for EPI in ("full", "c1", "bf16", "plain_bf16", "full", "c1"):
            print(EPI)
            measure(1)
