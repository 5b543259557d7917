"""How much of a class-A GEMM launch (the ResBlock convs of the VQ-VAE step) would overlap with a following
launch if tiles of consecutive problems shared one launch: the same call at M = 16384 (one wave of tiles, the
bench shape), 32768 and 65536 tokens (two and four waves, the later waves' main loops starting while the earlier
waves' epilogues stream).  usage on the GPU box: python tools/probe/classa_waves.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main(iters=20):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import kernels as K
    H, S = 512, 16
    bf, f32 = torch.bfloat16, torch.float32
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s, dt=bf: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(dt)  # noqa: E731
    Wf, Wd, We = r(H, 3 * H), r(3 * H, H), r(H, H)
    bias = r(H, dt=f32)
    seed = torch.zeros(1, dtype=torch.int64, device="cuda")
    conv, dconv = (H, S, 1, 0), (H, S, -1, 0)

    def cases(N):
        a, a1 = r(N, H), r(N, H)
        resid, pre32, pre16 = r(N, H, dt=f32), r(N, H, dt=f32), r(N, H)
        o32, o16, p16 = torch.empty(N, H, device="cuda"), torch.empty(N, H, device="cuda", dtype=bf), \
            torch.empty(N, H, device="cuda", dtype=bf)
        return [
            ("dec conv1 fwd", lambda: K.gemm(a, Wf, N, H, 3 * H, conv=conv, bias=bias, C=o16, C2=p16, c2_mode=1)),
            ("dec conv2 fwd", lambda: K.gemm(a1, Wf, N, H, 3 * H, conv=conv, bias=bias, drop=(0.1, 7), seed_ptr=seed,
                                             resid=resid, C=o32, C2=p16, c2_mode=1)),
            ("dec dgrad2", lambda: K.gemm(a, Wd, N, H, 3 * H, b_trans=True, conv=dconv, pre=pre16, C=o16)),
            ("dec dgrad1", lambda: K.gemm(a, Wd, N, H, 3 * H, b_trans=True, conv=dconv, pre=pre32, resid=resid, C=o32,
                                          C2=p16, c2_mode=3, drop2=(0.1, 9), seed_ptr=seed)),
            ("enc conv1 fwd", lambda: K.gemm(a, We, N, H, H, bias=bias, C=o16, C2=p16, c2_mode=1)),
            ("enc conv2 fwd", lambda: K.gemm(a1, We, N, H, H, bias=bias, drop=(0.1, 7), seed_ptr=seed, resid=resid,
                                             C=o32, C2=p16, c2_mode=1)),
            ("enc dgrad2", lambda: K.gemm(a, We, N, H, H, b_trans=True, pre=pre16, C=o16)),
            ("enc dgrad1", lambda: K.gemm(a, We, N, H, H, b_trans=True, pre=pre32, resid=resid, C=o32, C2=p16,
                                          c2_mode=3, drop2=(0.1, 9), seed_ptr=seed)),
        ]

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
        return t0.elapsed_time(t1) / iters * 1e3

    res = {}
    for N in (16384, 32768, 65536):
        for name, fn in cases(N):
            res.setdefault(name, []).append(timeit(fn))
        torch.cuda.empty_cache()
    print(f"{'launch':16s} {'M=16384':>9s} {'M=32768':>9s} {'M=65536':>9s}   per-wave cost at 2 / 4 waves", flush=True)
    for name, (t1, t2, t4) in res.items():
        print(f"{name:16s} {t1:9.1f} {t2:9.1f} {t4:9.1f}   {t2 / 2 / t1:5.2f} / {t4 / 4 / t1:5.2f}", flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
