"""The fused ResBlock chains (csrc/reschain.hip) alone at the configs[1] shape (N = 16384 tokens, H = 512, R = 8,
dropout 0.1): time per launch of aw_res_chain_fwd / aw_res_chain_bwd against the 2R per-conv aw_gemm launches each
replaces (the same epilogues), HIP events around `iters` launches after 3 warm-up ones; taps 1 = the encoder stack,
3 = the decoder's k = 3 stack.
usage on the GPU box: python tools/probe/res_chain_probe.py [iters] [taps]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main(iters=20, taps=1, N=16384):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import kernels as K
    H, R, p = 512, 8, 0.1
    TH = taps * H
    BF = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s, sc=1.0, dt=BF: (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)  # noqa: E731
    e = lambda: torch.empty(N, H, device="cuda", dtype=BF)  # noqa: E731
    a0, x0 = rnd(N, H), rnd(N, H)
    w1 = [rnd(H, TH, sc=TH ** -0.5) for _ in range(R)]
    w2 = [rnd(H, TH, sc=TH ** -0.5) for _ in range(R)]
    dg = lambda w: w.view(H, taps, H).permute(1, 0, 2).reshape(TH, H).contiguous()  # noqa: E731
    d1, d2 = [dg(w) for w in w1], [dg(w) for w in w2]
    b1 = [rnd(H, sc=0.1, dt=torch.float32) for _ in range(R)]
    b2 = [rnd(H, sc=0.1, dt=torch.float32) for _ in range(R)]
    seeds = list(range(1, R + 1))
    ctr = torch.ones(1, device="cuda", dtype=torch.int64)
    h, a1, x, a = [e() for _ in range(R)], [e() for _ in range(R)], [e() for _ in range(R - 1)] + [None], \
        [e() for _ in range(R)]
    wt = [torch.empty(H, TH, device="cuda", dtype=BF) for _ in range(2 * R)]
    pk = [torch.empty(H, TH, device="cuda", dtype=BF) for _ in range(2 * R)]
    gh, go = [e() for _ in range(R)], [e() for _ in range(R)]
    gx, gxo = rnd(N, H, sc=0.01), rnd(N, H, sc=0.01)
    xs = [x0] + x[:R - 1]
    masks = K.res_dropout_masks_empty(N, R, "cuda")
    fw = dict(conv=(H, 16, 1, 0)) if taps == 3 else {}
    bw = dict(conv=(H, 16, -1, 0)) if taps == 3 else {}

    def chain_fwd():
        K.res_chain_fwd(a0, x0, pk[:R], pk[R:], b1, b2, h, a1, x, a, drop=(p, seeds), seed_ptr=ctr, masks=masks,
                        taps=taps)

    def chain_bwd():
        K.res_chain_bwd(gx, gxo, wt[:R], wt[R:], h, x0, [None] + x[:R - 1], gh, go, drop_p=p, masks=masks, taps=taps)

    def pack():
        K.res_pack_weights(w1 + w2, pk, wt, taps=taps)

    def unfused_fwd():
        xr, ar = x0, a0
        for r in range(R):
            K.gemm(ar, w1[r], N, H, TH, bias=b1[r], C=h[r], C2=a1[r], c2_mode=1, **fw)
            if r < R - 1:
                K.gemm(a1[r], w2[r], N, H, TH, bias=b2[r], drop=(p, seeds[r]), seed_ptr=ctr, resid=xr, C=x[r],
                       C2=a[r], c2_mode=1, **fw)
                xr, ar = x[r], a[r]
            else:
                K.gemm(a1[r], w2[r], N, H, TH, bias=b2[r], drop=(p, seeds[r]), seed_ptr=ctr, resid=xr, C=a[r], **fw)

    def unfused_bwd():
        g_x, g_o = gx, gxo
        for r in reversed(range(R)):
            K.gemm(g_o, d2[r], N, H, TH, b_trans=True, pre=h[r], C=gh[r], **bw)
            K.gemm(gh[r], d1[r], N, H, TH, b_trans=True, pre=xs[r], resid=g_x, C=x[r] if r < R - 1 else a[r],
                   C2=go[r], c2_mode=3 if r > 0 else 2, drop2=(p, seeds[r - 1] if r > 0 else 0), seed_ptr=ctr, **bw)
            g_x, g_o = (x[r] if r < R - 1 else a[r]), go[r]

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(iters):
            fn()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) * 1000.0 / iters

    fl = 4.0 * R * N * H * H * (1 if taps == 1 else 3 - 2 / 16)
    from arcweld import vqvae  # noqa: F401
    print(f"taps {taps}", flush=True)
    with K.store_policy(1):
        for name, fn in (("chain_fwd", chain_fwd), ("unfused_fwd", unfused_fwd), ("pack", pack),
                         ("chain_bwd", chain_bwd), ("unfused_bwd", unfused_bwd)):
            us = timeit(fn)
            tf = fl / (us * 1e-6) / 1e12 if "pack" not in name else 0.0
            print(f"{name:12s} {us:8.1f} us   {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main(*(int(v) for v in sys.argv[1:]))
