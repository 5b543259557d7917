"""Can an MFMA-bound weight-gradient GEMM stream fill the MFMA-idle epilogue phases of an epilogue-heavy GEMM chain?
Stream 1: `depth` decoder-conv launches (M 16384, N 512, K 1536 implicit conv, full residual/dropout epilogue),
each dependent on the previous.  Stream 2: `depth` weight-gradient launches (512 x 1536 x 16384, accumulate).
Timed alone and forked together inside one captured graph.  usage: python tools/probe/stream_overlap.py"""
import sys

import torch

sys.path.insert(0, "vq-vae-transformer-arc-welding_amd")
from arcweld import kernels as K  # noqa: E402

H, S, depth, M = 512, 16, 16, 16384


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    y = [torch.randn(M, H, device="cuda", generator=g) for _ in range(2)]
    a = [torch.randn(M, H, device="cuda", generator=g).bfloat16() for _ in range(2)]
    W = (torch.randn(H, 3 * H, device="cuda", generator=g) * 0.02).bfloat16()
    bias = torch.zeros(H, device="cuda")
    ctr = torch.zeros(1, device="cuda", dtype=torch.int64)
    go = torch.randn(M, H, device="cuda", generator=g).bfloat16()
    acts = [torch.randn(M, H, device="cuda", generator=g).bfloat16() for _ in range(depth)]
    gw = torch.zeros(H, 3 * H, device="cuda")

    We = (torch.randn(H, H, device="cuda", generator=g) * 0.02).bfloat16()

    def chain():      # encoder-backward-like: K = 512 input-gradient launches with GELU' + residual epilogues
        for i in range(depth):
            src, dst = i % 2, (i + 1) % 2
            K.gemm(a[src], We, M, H, H, b_trans=True, pre=y[src], resid=y[dst], C=y[src], C2=a[dst], c2_mode=3,
                   drop2=(0.1, 77 + i), seed_ptr=ctr)

    def wgrads():     # the decoder's deferred weight gradients: one grouped launch
        K.gemm_grouped([(go, acts[i], H, 3 * H, M, dict(a_trans=True, b_trans=True, conv=(H, S, 1, 1),
                                                        C=gw.view(H, 3 * H), accumulate=True, col_map=(H, 3, 0)))
                        for i in range(depth)])

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def body(which):
        main = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(main)
        for s in (s1, s2):
            s.wait_event(ev)
        if which in ("chain", "both"):
            with torch.cuda.stream(s1):
                chain()
        if which in ("wgrad", "both"):
            with torch.cuda.stream(s2):
                wgrads()
        if which == "serial":
            with torch.cuda.stream(s1):
                chain()
                wgrads()
        for s in (s1, s2):
            e = torch.cuda.Event()
            e.record(s)
            main.wait_event(e)

    for which in ("chain", "wgrad", "serial", "both", "chain", "wgrad", "serial", "both"):
        body(which)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            body(which)
        for _ in range(3):
            gr.replay()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            gr.replay()
        t1.record()
        torch.cuda.synchronize()
        print(f"{which:7s} {t0.elapsed_time(t1) / 10 * 1e3:9.1f} us", flush=True)


if __name__ == "__main__":
    main()
