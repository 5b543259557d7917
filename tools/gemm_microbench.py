"""GEMM micro-benchmark on the GPU: time one aw_gemm shape while toggling epilogue features / K, to attribute
time between the MFMA main loop and the epilogue.  Usage: python tools/gemm_microbench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
import torch  # noqa: E402

from arcweld import kernels as K  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def run():
    M, N, H = 16384, 512, 512
    A3 = torch.randn(M, 3 * H, device=dev).to(bf)
    A = A3[:, :H].contiguous()
    W = torch.randn(N, H, device=dev).to(bf)
    W3 = torch.randn(N, 3 * H, device=dev).to(bf)
    C = torch.empty(M, N, device=dev)
    C2 = torch.empty(M, N, device=dev, dtype=bf)
    Cb = torch.empty(M, N, device=dev, dtype=bf)
    pre = torch.randn(M, N, device=dev)
    res = torch.randn(M, N, device=dev)
    bias = torch.randn(N, device=dev)
    rows = []

    def rec(name, us, flops, bytes_):
        rows.append((name, us, flops / us / 1e6, bytes_ / us / 1e3))

    fl = 2 * M * N * H
    rec("K512 C f32", timeit(lambda: K.gemm(A, W, M, N, H, C=C)), fl, M * H * 2 + M * N * 4)
    rec("K512 C bf16", timeit(lambda: K.gemm(A, W, M, N, H, C=Cb)), fl, M * H * 2 + M * N * 2)
    rec("K512 C f32 + C2 gelu", timeit(lambda: K.gemm(A, W, M, N, H, bias=bias, C=C, C2=C2, c2_mode=1)), fl,
        M * H * 2 + M * N * 6)
    rec("K512 full bwd epi", timeit(lambda: K.gemm(A, W, M, N, H, pre=pre, resid=res, C=C, C2=C2, c2_mode=3,
                                                    drop2=(0.1, 7))), fl, M * H * 2 + M * N * 14)
    rec("K512 b_trans C f32", timeit(lambda: K.gemm(A, W, M, N, H, b_trans=True, C=C)), fl, M * H * 2 + M * N * 4)
    fl3 = 2 * M * N * 3 * H
    rec("K1536 C f32", timeit(lambda: K.gemm(A3, W3, M, N, 3 * H, C=C)), fl3, M * 3 * H * 2 + M * N * 4)
    rec("K1536 conv C f32", timeit(lambda: K.gemm(A, W3, M, N, 3 * H, conv=(H, 16, 1, 0), C=C)), fl3,
        M * H * 2 + M * N * 4)
    rec("K1536 conv + gelu", timeit(lambda: K.gemm(A, W3, M, N, 3 * H, conv=(H, 16, 1, 0), bias=bias, C=C, C2=C2,
                                                    c2_mode=1)), fl3, M * H * 2 + M * N * 6)
    A8 = torch.randn(M, 4096, device=dev).to(bf)
    W8 = torch.randn(N, 4096, device=dev).to(bf)
    rec("K4096 C f32", timeit(lambda: K.gemm(A8, W8, M, N, 4096, C=C)), 2 * M * N * 4096, M * 4096 * 2 + M * N * 4)
    Wb = torch.randn(4096, 4096, device=dev).to(bf)
    Ab = torch.randn(4096, 4096, device=dev).to(bf)
    Cbig = torch.empty(4096, 4096, device=dev)
    rec("4096^3 C f32", timeit(lambda: K.gemm(Ab, Wb, 4096, 4096, 4096, C=Cbig)), 2 * 4096 ** 3, 3 * 4096 * 4096 * 4)
    G = torch.zeros(N, H, 3, device=dev)
    rec("wgrad 512x512xK16384", timeit(lambda: K.gemm(A, A, H, H, M, a_trans=True, b_trans=True,
                                                      C=G.view(H, 3 * H), accumulate=True, col_map=(0, 3, 1))),
        2 * M * H * H, 2 * M * H * 2)
    print(f"{'case':28s} {'us':>9s} {'TFLOP/s':>9s} {'GB/s':>9s}")
    for r in rows:
        print(f"{r[0]:28s} {r[1]:9.1f} {r[2]:9.1f} {r[3]:9.1f}")


if __name__ == "__main__" and len(sys.argv) == 1:
    run()


def sweep():
    """K sweep at M=16384, N=512 (C f32 only / no output at all via C bf16 tiny?): run under rocprofv3 to get pure
    kernel durations; python tools/gemm_microbench.py sweep"""
    M, N = 16384, 512
    for Kd in (64, 128, 256, 512, 1024, 2048):
        A = torch.randn(M, Kd, device=dev).to(bf)
        W = torch.randn(N, Kd, device=dev).to(bf)
        C = torch.empty(M, N, device=dev)
        Cb = torch.empty(M, N, device=dev, dtype=bf)
        t1 = timeit(lambda: K.gemm(A, W, M, N, Kd, C=C))
        t2 = timeit(lambda: K.gemm(A, W, M, N, Kd, C=Cb))
        print(f"K={Kd:5d}  C f32 {t1:7.1f} us   C bf16 {t2:7.1f} us", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sweep":
    sweep()
