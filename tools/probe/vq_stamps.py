"""Where the VQ forward kernel (vq_fwd_kernel, configs[1] shape N 16384, K 512 x D 64: 512 workgroups of 32 rows)
spends its time: per-workgroup s_memrealtime stamps (100 MHz) from a probe build with -DAW_VQ_STAMPS at entry (0),
after the z tile (1), after the first codebook chunk is in LDS (2), after each codebook step (3..), after the
cross-wave argmin exchange (11) and at the end of wave 0's epilogue (12).  Build on the CPU first:
  make -C vq-vae-transformer-arc-welding_amd/csrc -j8 OUT=../../tools/probe/build/libarcweld_vqstamps.so \\
       OBJDIR=../../tools/probe/build/obj_vqstamps EXTRA=-DAW_VQ_STAMPS
usage on the GPU box: python tools/probe/vq_stamps.py"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "build", "libarcweld_vqstamps.so")


def main(N=16384, Kc=512, D=64, iters=20):
    os.environ["ARCWELD_LIB"] = LIB
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import _native
    from arcweld import kernels as K
    lib = _native.load()
    print("library:", _native.LIB_PATH, flush=True)
    rd = lib.aw_probe_vq_stamps
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    g = torch.Generator(device="cuda").manual_seed(0)
    z = torch.randn(N, D, device="cuda", generator=g) * 0.08
    E = torch.randn(Kc, D, device="cuda", generator=g) * 0.08
    zq = torch.empty_like(z)
    zq2 = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
    idx = torch.empty(N, dtype=torch.int64, device="cuda")
    counts = torch.zeros(Kc, device="cuda")
    sq = torch.zeros(1, device="cuda", dtype=torch.float64)
    fn = lambda: K.vq_forward(z, E, zq, idx, counts, sq, zq_copy=zq2)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        fn()
    t1.record()
    torch.cuda.synchronize()
    print(f"N {N} K {Kc} D {D}: {t0.elapsed_time(t1) / iters * 1e3:.1f} us/launch", flush=True)
    NW = 1024 * 16
    buf = (ctypes.c_uint64 * NW)()
    for rep in range(3):
        rd(buf, NW)
        fn()
        torch.cuda.synchronize()
        assert rd(buf, NW) == NW
        st = [[buf[b * 16 + i] for i in range(16)] for b in range(1024)]
        st = [s for s in st if s[0] and s[12]]
        base = min(s[0] for s in st)
        end = max(s[12] for s in st)
        med = lambda xs: statistics.median(xs) / 100.0  # noqa: E731  (10 ns ticks -> us)
        mx = lambda xs: max(xs) / 100.0  # noqa: E731
        steps = [i for i in range(3, 11) if all(s[i] for s in st)]
        names = [("z tile", 0, 1), ("zz+chunk0", 1, 2)]
        prev = 2
        for i in steps:
            names.append((f"step{i - 3}", prev, i))
            prev = i
        names += [("argmin xchg", prev, 11), ("wave0 epi", 11, 12)]
        print(f"rep {rep}: {len(st)} wgs, start spread {(max(s[0] for s in st) - base) / 100:.1f} us, "
              f"first start -> last end {(end - base) / 100:.1f} us", flush=True)
        print("   phase          median    max  (us)")
        for nm, a, b in names:
            d = [s[b] - s[a] for s in st]
            print(f"   {nm:12s} {med(d):7.2f} {mx(d):7.2f}")
        tot = [s[12] - s[0] for s in st]
        print(f"   {'total':12s} {med(tot):7.2f} {mx(tot):7.2f}", flush=True)


if __name__ == "__main__":
    main()
