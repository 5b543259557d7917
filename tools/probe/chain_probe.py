"""Timing probe of the fused encoder chain (aw_encoder_chain_fwd) at the configs[1] shape (N 16384 tokens, H 512,
R 8): the library kernel against variants built with EC_PROBE / EC_AUX settings (csrc/encoder_chain.hip header: e.g.
"1" no overlapped stores, "5" no stores and no MFMA, "0:0" default-policy stores) and the 16 per-block aw_gemm
launches it replaces.
Build the variants on the CPU first:  python tools/probe/chain_probe.py build ;  then on the GPU:  python
tools/probe/chain_probe.py"""
import ctypes
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd")]
CSRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
OUT = os.path.join(REPO, "tools", "probe", "build")
# "probe" or "probe:aux" (EC_AUX = the store cache-policy bits)
VARIANTS = os.environ.get("EC_VARIANTS", "1,0:0,5").split(",")


def _defs(v):
    p, _, aux = v.partition(":")
    return [f"-DEC_PROBE={p}"] + ([f"-DEC_AUX={aux}"] if aux else [])


def build():
    os.makedirs(OUT, exist_ok=True)
    for v in VARIANTS:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
               *_defs(v), f"-I{os.path.join(REPO, 'include')}", os.path.join(CSRC, "encoder_chain.hip"),
               os.path.join(CSRC, "runtime.hip"), "-o", os.path.join(OUT, f"chain_{v.replace(':', '_')}.so")]
        subprocess.run(cmd, check=True)


def main():
    import torch
    from arcweld import _native as nat
    from arcweld import kernels as K
    N, H, R = 16384, 512, 8
    g = torch.Generator(device="cuda").manual_seed(0)
    W = [(torch.randn(H, H, device="cuda", generator=g) * 0.04).bfloat16() for _ in range(2 * R)]
    b = [torch.randn(H, device="cuda", generator=g) * 0.1 for _ in range(2 * R)]
    x0 = torch.randn(N, H, device="cuda", generator=g)
    a0 = torch.nn.functional.gelu(x0).bfloat16()
    e = lambda dt=torch.bfloat16: torch.empty(N, H, device="cuda", dtype=dt)  # noqa: E731
    hs, a1s, xs, aos = [e() for _ in range(R)], [e() for _ in range(R)], [e(torch.float32) for _ in range(R)], \
        [e() for _ in range(R)]
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")

    Wx = [w.view(H, 16, 32).transpose(0, 1).contiguous() for w in W]   # the chain's K-step-major copies

    def args(p):
        a = nat.EncoderChainArgs()
        a.N, a.H, a.R = N, H, R
        a.x0, a.a0 = x0.data_ptr(), a0.data_ptr()
        a.drop_p = p
        for r in range(R):
            a.W1[r], a.W2[r], a.b1[r], a.b2[r] = (Wx[2 * r].data_ptr(), Wx[2 * r + 1].data_ptr(), b[2 * r].data_ptr(),
                                                  b[2 * r + 1].data_ptr())
            a.drop_seed[r] = 1234 + r
            a.h[r], a.a1[r], a.x[r], a.aout[r] = (hs[r].data_ptr(), a1s[r].data_ptr(), xs[r].data_ptr(),
                                                  aos[r].data_ptr())
        a.seed_ptr = ctr.data_ptr()
        return a

    def timeit(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) / iters * 1e3

    flop = 2.0 * N * H * H * 2 * R
    so = lambda v: os.path.join(OUT, f"chain_{v.replace(':', '_')}.so")  # noqa: E731
    libs = [("library", nat.load())] + [(f"EC_PROBE={v}", ctypes.CDLL(so(v))) for v in VARIANTS
                                       if os.path.exists(so(v))]
    stream = torch.cuda.current_stream().cuda_stream
    for p in (0.0, 0.1):
        for name, lib in libs:
            a = args(p)
            us = timeit(lambda: lib.aw_encoder_chain_fwd(ctypes.byref(a), ctypes.c_void_p(stream)))
            print(f"p={p} {name:12s} {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)

    def per_block():
        x, a = x0, a0
        for r in range(R):
            K.gemm(a, W[2 * r], N, H, H, bias=b[2 * r], C=hs[r], C2=a1s[r], c2_mode=1)
            K.gemm(a1s[r], W[2 * r + 1], N, H, H, bias=b[2 * r + 1], resid=x, C=xs[r], C2=aos[r], c2_mode=1)
            x, a = xs[r], aos[r]
    try:
        us = timeit(per_block)
        print(f"per-block aw_gemm x{2 * R}: {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)
    except Exception as ex:           # the probe's per-block call shape may drift from kernels.gemm
        print("per-block timing skipped:", ex)


if __name__ == "__main__":
    build() if sys.argv[1:] == ["build"] else main()
