"""The transformer's grouped weight-gradient launches (arcweld/decoder.py: per layer kind, 4 blocks per launch, token
reduction R = 51 x 321 = 16,371, bf16 operands token-major) under the 128-row tile (automatic policy) and the 256-row
ping-pong tile (aw_gemm_set_tile(256)), with the library in ARCWELD_LIB (e.g. a build whose grouped split-K cap,
AW_GROUPED_MAXSPLIT, differs).  usage on the GPU box: [ARCWELD_LIB=...] python tools/probe/twgrad_probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main(iters=10):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import _native
    from arcweld import kernels as K
    d, R, G = 512, 51 * 321, 4
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(bf)  # noqa: E731
    kinds = {"fc2 (512 x 2048)": (d, 4 * d), "fc1 (2048 x 512)": (4 * d, d), "proj (512 x 512)": (d, d),
             "qkv (1536 x 512)": (3 * d, d)}

    def probs(M, N):
        out = []
        for _ in range(G):
            A, B = r(R, M), r(R, N)
            C, rs = torch.zeros(M, N, device="cuda"), torch.zeros(M, device="cuda")
            out.append((A, B, M, N, R, dict(a_trans=True, b_trans=True, C=C, accumulate=True, a_rowsum=rs)))
        return out

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

    print("library:", _native.LIB_PATH, flush=True)
    total = {0: 0.0, 256: 0.0}
    for name, (M, N) in kinds.items():
        p = probs(M, N)
        ref = None
        line = f"{name:18s}"
        for tile in (0, 256):
            _native.call("aw_gemm_set_tile", tile)
            for (_, _, _, _, _, kw) in p:
                kw["C"].zero_()
            K.gemm_grouped(p)
            torch.cuda.synchronize()
            got = torch.stack([kw["C"] for (*_, kw) in p])
            if ref is None:
                ref = got.clone()
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            us = timeit(lambda: K.gemm_grouped(p))
            total[tile] += us
            fl = G * 2.0 * M * N * R
            line += f"  tile {tile or 'auto'}: {us:7.1f} us ({fl / us / 1e6:6.1f} TF, rel.diff {err:.1e})"
        print(line, flush=True)
    _native.call("aw_gemm_set_tile", 0)
    print(f"sum of the 4 kinds: auto {total[0]:.1f} us, tile 256 {total[256]:.1f} us", flush=True)


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
