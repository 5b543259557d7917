"""Library GEMM reference points on the box (hipBLASLt via torch.matmul, bf16): the same shapes as the VQ-VAE
step's launches, to price our kernels against the vendor library.  usage: python tools/probe/torch_gemm_ref.py"""
import torch

SHAPES = [  # (name, M, N, K, batch)
    ("enc fwd 16384x512x512", 16384, 512, 512, 1),
    ("dec fwd 16384x512x1536", 16384, 512, 1536, 1),
    ("dec wgrad 512x1536x16384", 512, 1536, 16384, 1),
    ("dec wgrad x16 grouped (bmm)", 512, 1536, 16384, 16),
    ("enc wgrad x16 grouped (bmm)", 512, 512, 16384, 16),
    ("convT1 16384x2560x512", 16384, 2560, 512, 1),
    ("big 8192^3", 8192, 8192, 8192, 1),
]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    torch.manual_seed(0)
    for name, M, N, K, b in SHAPES:
        if b == 1:
            a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
            us = bench(lambda: torch.matmul(a, w))
        else:
            # weight-gradient shape: [M, K] x [K, N] with the token axis K as the reduction
            a = torch.randn(b, K, M, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
            w = torch.randn(b, K, N, device="cuda", dtype=torch.bfloat16)
            us = bench(lambda: torch.bmm(a, w))
        tf = 2.0 * M * N * K * b / us / 1e6
        print(f"{name:34s} {us:9.1f} us  {tf:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
