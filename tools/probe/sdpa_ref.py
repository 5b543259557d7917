"""Reference point only (not the product path): torch's fused scaled_dot_product_attention on ROCm at the transformer
bench shape (51 x 8 heads x 321 x 64, bf16, causal), forward and forward+backward, timed with HIP events.
usage: python tools/probe/sdpa_ref.py"""
import torch
import torch.nn.functional as F

B, H, T, D = 51, 8, 321, 64


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B, H, T, D, device="cuda", generator=g).bfloat16().requires_grad_() for _ in range(3))
    do = torch.randn(B, H, T, D, device="cuda", generator=g).bfloat16()
    for backend in ("FLASH_ATTENTION", "EFFICIENT_ATTENTION", "MATH"):
        be = getattr(torch.nn.attention.SDPBackend, backend)
        try:
            with torch.nn.attention.sdpa_kernel(be):
                fwd = timed(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True))
                out = F.scaled_dot_product_attention(q, k, v, is_causal=True)
                fb = timed(lambda: torch.autograd.grad(F.scaled_dot_product_attention(q, k, v, is_causal=True),
                                                       (q, k, v), do))
            print(f"{backend}: fwd {fwd:.1f} us, fwd+bwd {fb:.1f} us", flush=True)
        except Exception as e:   # backend unavailable on this build
            print(f"{backend}: unavailable ({type(e).__name__}: {str(e)[:100]})", flush=True)


if __name__ == "__main__":
    main()
