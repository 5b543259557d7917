"""The stream-K batched weight-gradient kernel (csrc/wgrad.hip, wgrad_tt_kernel) alone: time per launch at the
transformer's half-step batch (4 blocks x {qkv, proj, fc1, fc2} at d 512, K = 51 x 321 tokens) and at the VQ-VAE
encoder's 16 centre-tap convs (512 x 512, K 16384), for the library kernel and probe builds with parts left out
(WT_NO_FIX: split pieces neither published nor summed; WT_SKIP_DMA / WT_SKIP_READS / WT_SKIP_MFMA; results of the probe
builds are garbage by construction).  Build on the CPU first:  python tools/probe/wgrad_tt_probe.py build
usage on the GPU box: python tools/probe/wgrad_tt_probe.py [iters]"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
VARIANTS = {"base": [], "no_fix": ["-DWT_NO_FIX"], "skip_dma": ["-DWT_SKIP_DMA"], "skip_reads": ["-DWT_SKIP_READS"],
            "skip_mfma": ["-DWT_SKIP_MFMA"], "skip_dma_reads": ["-DWT_SKIP_DMA", "-DWT_SKIP_READS"],
            "mfma_only": ["-DWT_SKIP_DMA", "-DWT_SKIP_READS", "-DWT_NO_FIX"]}


def build():
    procs = []
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    for name, flags in VARIANTS.items():
        out = os.path.join(HERE, "build", f"wt_{name}.so")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wl,-Bsymbolic",
               "-munsafe-fp-atomics", "-DWT_PROBE", *flags, "-I" + os.path.join(REPO, "include"),
               os.path.join(SRC, "wgrad.hip"), os.path.join(SRC, "runtime.hip"), "-o", out]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0


def problems(case, torch, K):
    g = torch.Generator(device="cuda").manual_seed(0)
    d = 512
    if case == "transformer_half":
        Kt, shapes = 51 * 321, [(3 * d, d), (d, d), (4 * d, d), (d, 4 * d)] * 4
    else:
        Kt, shapes = 16384, [(d, d)] * 16
    out = []
    for M, N in shapes:
        A = torch.randn(Kt, M, device="cuda", generator=g).bfloat16()
        B = torch.randn(Kt, N, device="cuda", generator=g).bfloat16()
        out.append((A, B, M, N, Kt, dict(a_trans=True, b_trans=True, C=torch.zeros(M, N, device="cuda"),
                                         accumulate=True, a_rowsum=torch.zeros(M, device="cuda"))))
    return out


def main(iters=10):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import kernels as K
    from arcweld import _native

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

    for case in ("transformer_half", "encoder"):
        probs = problems(case, torch, K)
        fl = sum(2.0 * M * N * Kd for (_, _, M, N, Kd, _) in probs)
        arr = (K.GemmArgs * len(probs))(*[K._gemm_args(a, b, M, N, Kd, **kw) for (a, b, M, N, Kd, kw) in probs])
        lib = _native.load()
        wsb = lib.aw_wgrad_batch_workspace(arr, len(probs))
        ws = torch.empty(wsb // 4, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        res = {"generic_grouped": timeit(lambda: [K.gemm_grouped([p for p in probs if (p[2], p[3]) == sh])
                                                  for sh in dict.fromkeys((p[2], p[3]) for p in probs)])}
        for name in VARIANTS:
            pl = ctypes.CDLL(os.path.join(HERE, "build", f"wt_{name}.so"))
            fn = pl.wt_probe_batch
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
            res[name] = timeit(lambda: fn(ctypes.cast(arr, ctypes.c_void_p), len(probs), ws.data_ptr(), wsb, s))
        print(case, " ".join(f"{k} {v:.1f}us ({fl / v / 1e6:.0f} TF)" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
