"""The decoder k = 3 weight-gradient kernel (csrc/wgrad.hip) alone at the VQ-VAE bench shape (16 convs, O = I = 512,
16384 tokens, windows of 16): time per launch of the library kernel, the generic grouped GEMM, and probe builds with
parts of the loop left out (W3_SKIP_DMA / W3_SKIP_READS / W3_SKIP_MFMA / W3_NO_STAGGER; results of those are
garbage by construction).  Build the probe libraries on the CPU first:  python tools/probe/wgrad3_probe.py build
usage on the GPU box: python tools/probe/wgrad3_probe.py [iters]"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
VARIANTS = {"base": [], "skip_dma": ["-DW3_SKIP_DMA"], "skip_reads": ["-DW3_SKIP_READS"],
            "skip_mfma": ["-DW3_SKIP_MFMA"], "skip_dma_reads": ["-DW3_SKIP_DMA", "-DW3_SKIP_READS"],
            "mask_in_m": ["-DW3_MASK_IN_M"], "no_prio": ["-DW3_NO_PRIO"], "sched2": ["-DW3_SCHED=2"],
            "sched0": ["-DW3_SCHED=0"], "stamps": ["-DW3_STAMPS"], "stamps_s2": ["-DW3_STAMPS", "-DW3_SCHED=2"]}


def build():
    procs = []
    for name, flags in VARIANTS.items():
        out = os.path.join(HERE, "build", f"w3_{name}.so")
        # -Bsymbolic: each probe library calls its OWN launcher (not the arcweld library's, loaded earlier)
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wl,-Bsymbolic",
               "-munsafe-fp-atomics", "-DW3_PROBE", *flags, "-I" + os.path.join(REPO, "include"),
               os.path.join(SRC, "wgrad.hip"), os.path.join(SRC, "runtime.hip"), "-o", out]
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        assert p.wait() == 0


def main(iters=10):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import _native
    from arcweld import kernels as K
    N, H, S, G = 16384, 512, 16, 16
    g = torch.Generator(device="cuda").manual_seed(0)
    A = [torch.randn(N, H, device="cuda", generator=g).bfloat16() for _ in range(G)]
    B = [torch.randn(N, H, device="cuda", generator=g).bfloat16() for _ in range(G)]
    C = [torch.zeros(H, 3 * H, device="cuda") for _ in range(G)]
    bias = [torch.zeros(H, device="cuda") for _ in range(G)]
    probs = [(A[i], B[i], H, 3 * H, N, dict(a_trans=True, b_trans=True, conv=(H, S, 1, 1), C=C[i], accumulate=True,
                                            a_rowsum=bias[i])) for i in range(G)]
    arr = (K.GemmArgs * G)(*[K._gemm_args(a, b, M, Nn, Kd, **kw) for (a, b, M, Nn, Kd, kw) in probs])
    fl = G * 2.0 * H * 3 * H * N

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

    s = torch.cuda.current_stream().cuda_stream
    rows = []
    for pol, name in ((-1, "library generic grouped GEMM"), (1, "library wgrad_conv3_kernel")):
        _native.call("aw_gemm_set_wgrad_policy", pol)
        rows.append((name, timeit(lambda: K.gemm_grouped(probs))))
    _native.call("aw_gemm_set_wgrad_policy", 0)
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(HERE, "build", f"w3_{name}.so"))
        lib.w3_probe_grouped.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]

        def run(lib=lib):
            assert lib.w3_probe_grouped(arr, G, ctypes.c_void_p(s)) == 0
        rows.append((f"probe {name}", timeit(run)))
    for sname in ("stamps", "stamps_s2"):
      lib = ctypes.CDLL(os.path.join(HERE, "build", f"w3_{sname}.so"))
      buf = (ctypes.c_uint64 * 384)()
      print(sname)
      if lib.w3_probe_stamps(buf, 384) == 384:
        # per (workgroup, group, K-tile): R issue, barrier wait, M, rowsum, barrier wait (cycles of s_memtime)
        segs = ("R", "bar1", "M", "post", "bar2")
        tot = {k: [] for k in segs}
        for wg in range(8):
            for grp in range(2):
                for t in range(4):
                    b = ((wg * 2 + grp) * 4 + t) * 6
                    v = [buf[b + k] for k in range(6)]
                    for k, name in enumerate(segs):
                        tot[name].append(v[k + 1] - v[k])
                    if wg < 1:
                        print(f"wg {wg} grp {grp} t {t}: " + " ".join(f"{n}={v[k + 1] - v[k]}" for k, n in enumerate(segs)))
        print("median cycles: " + " ".join(f"{n}={sorted(x)[len(x) // 2]}" for n, x in tot.items()), flush=True)
    for name, us in rows:
        print(f"{name:34s} {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  frac {fl / us / 1e6 / 2500:.3f}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
