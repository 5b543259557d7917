"""Where a class-A GEMM launch (M = 16384 tokens, N = 512; the ResBlock forward and input-gradient convs of the
VQ-VAE step) spends its time: per-workgroup s_memrealtime stamps (100 MHz) at kernel entry, after the prologue,
after the main loop, after the accumulator tile is in LDS and after the epilogue (gemm_core.h AW_STAMP), from a
probe build of the library with -DAW_GEMM_STAMPS.  Arguments are the ones arcweld/vqvae.py passes at the bench
shape (bf16 operands, dropout 0.1).  Build on the CPU first (csrc/Makefile):
  make -C vq-vae-transformer-arc-welding_amd/csrc -j8 OUT=../../tools/probe/build/libarcweld_stamps.so \\
       OBJDIR=../../tools/probe/build/obj_stamps EXTRA=-DAW_GEMM_STAMPS
usage on the GPU box: python tools/probe/classa_stamps.py"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
STAMPS_LIB = os.path.join(HERE, "build", "libarcweld_stamps.so")


def cases(torch, K):
    N, H, S = 16384, 512, 16
    g = torch.Generator(device="cuda").manual_seed(0)
    bf, f32 = torch.bfloat16, torch.float32
    r = lambda *s, dt=bf: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(dt)  # noqa: E731
    a, a1 = r(N, H), r(N, H)
    Wf, Wd = r(H, 3 * H), r(3 * H, H)          # decoder conv: forward [O][3I], input-gradient [3O][I]
    We = r(H, H)
    bias = r(H, dt=f32)
    resid, pre32 = r(N, H, dt=f32), r(N, H, dt=f32)
    pre16 = r(N, H)
    seed = torch.zeros(1, dtype=torch.int64, device="cuda")
    conv, dconv = (H, S, 1, 0), (H, S, -1, 0)
    e = lambda dt=f32: torch.empty(N, H, device="cuda", dtype=dt)  # noqa: E731
    return [
        ("dec conv1 fwd (bias, C bf16, C2 gelu)", lambda: K.gemm(a, Wf, N, H, 3 * H, conv=conv, bias=bias, C=e(bf),
                                                                   C2=e(bf), c2_mode=1)),
        ("dec conv2 fwd (bias, drop, resid, C f32, C2 gelu)",
         lambda: K.gemm(a1, Wf, N, H, 3 * H, conv=conv, bias=bias, drop=(0.1, 7), seed_ptr=seed, resid=resid,
                        C=e(), C2=e(bf), c2_mode=1)),
        ("dec dgrad2 (gelu' bf16 pre, C bf16)", lambda: K.gemm(a, Wd, N, H, 3 * H, b_trans=True, conv=dconv,
                                                               pre=pre16, C=e(bf))),
        ("dec dgrad1 (gelu' f32 pre, resid, C f32, C2 drop)",
         lambda: K.gemm(a, Wd, N, H, 3 * H, b_trans=True, conv=dconv, pre=pre32, resid=resid, C=e(), C2=e(bf),
                        c2_mode=3, drop2=(0.1, 9), seed_ptr=seed)),
        ("enc conv1 fwd (bias, C bf16, C2 gelu)", lambda: K.gemm(a, We, N, H, H, bias=bias, C=e(bf), C2=e(bf),
                                                                   c2_mode=1)),
        ("enc conv2 fwd (bias, drop, resid, C f32, C2 gelu)",
         lambda: K.gemm(a1, We, N, H, H, bias=bias, drop=(0.1, 7), seed_ptr=seed, resid=resid, C=e(), C2=e(bf),
                        c2_mode=1)),
        ("enc dgrad2 (gelu' bf16 pre, C bf16)", lambda: K.gemm(a, We, N, H, H, b_trans=True, pre=pre16, C=e(bf))),
        ("enc dgrad1 (gelu' f32 pre, resid, C f32, C2 drop)",
         lambda: K.gemm(a, We, N, H, H, b_trans=True, pre=pre32, resid=resid, C=e(), C2=e(bf), c2_mode=3,
                        drop2=(0.1, 9), seed_ptr=seed)),
        ("plain K1536 (C bf16 only)", lambda: K.gemm(a, Wd.view(H, 3 * H), N, H, 3 * H, C=e(bf))),
    ]


def main(iters=20):
    stamps = os.path.exists(STAMPS_LIB) and os.environ.get("NO_STAMPS") != "1"
    if stamps:
        os.environ["ARCWELD_LIB"] = STAMPS_LIB
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import _native
    from arcweld import kernels as K
    lib = _native.load()
    print("library:", _native.LIB_PATH, flush=True)
    readers = []
    if stamps:
        for nm in ("aw_probe_stamps_256", "aw_probe_stamps_fwd", "aw_probe_stamps_bwd"):
            f = getattr(lib, nm)
            f.argtypes = [ctypes.c_void_p, ctypes.c_int]
            readers.append(f)
    NW = 8192 * 8
    buf = (ctypes.c_uint64 * NW)()
    for name, fn in cases(torch, K):
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
        line = f"{name:52s} {us:7.1f} us/launch"
        if stamps:
            for rd in readers:
                rd(buf, NW)                       # clear
            fn()
            torch.cuda.synchronize()
            for rd in readers:
                assert rd(buf, NW) == NW
                st = [tuple(buf[b * 8 + i] for i in range(5)) for b in range(8192)]
                st = [s for s in st if s[0] and s[4]]
                if st:
                    break
            if st:
                base = min(s[0] for s in st)
                med = lambda xs: statistics.median(xs) / 100.0  # noqa: E731  (ticks of 10 ns -> us)
                line += (f" | {len(st)} wgs: start spread {(max(s[0] for s in st) - base) / 100:5.1f}, end "
                         f"{(max(s[4] for s in st) - base) / 100:5.1f}; median prologue {med([s[1] - s[0] for s in st]):5.2f}"
                         f" loop {med([s[2] - s[1] for s in st]):5.2f} tile->LDS {med([s[3] - s[2] for s in st]):5.2f}"
                         f" epilogue {med([s[4] - s[3] for s in st]):5.2f} us")
                # per XCD (blocks b, b + 8, ... share one; s_memrealtime may be offset between XCDs): start spread
                # and first-start -> last-end span of the XCD's workgroups
                idx = [b for b in range(8192) if buf[b * 8] and buf[b * 8 + 4]]
                per = {}
                for b in idx:
                    per.setdefault(b % 8, []).append(tuple(buf[b * 8 + i] for i in range(5)))
                line += "\n    per XCD start spread / span (us): " + " ".join(
                    f"{(max(x[0] for x in v) - min(x[0] for x in v)) / 100:.1f}/"
                    f"{(max(x[4] for x in v) - min(x[0] for x in v)) / 100:.1f}" for _, v in sorted(per.items()))
                # how many workgroups are in their epilogue at each moment (1 us bins)
                span = max(s[4] for s in st) - base
                bins = [0] * (span // 100 + 1)
                loop = [0] * (span // 100 + 1)
                for s in st:
                    for t in range((s[3] - base) // 100, (s[4] - base) // 100 + 1):
                        bins[t] += 1
                    for t in range((s[1] - base) // 100, (s[2] - base) // 100 + 1):
                        loop[t] += 1
                line += "\n    in main loop per us: " + " ".join(str(v) for v in loop)
                line += "\n    in epilogue  per us: " + " ".join(str(v) for v in bins)
        print(line, flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
