"""Probe builds of csrc/reschain.hip (EC_PROBE_FLAGS, see the top of that file): the chain kernels alone at the
configs[1] shape with parts left out, and per-conv s_memtime stamps.  Results of the probe builds are garbage by
construction.  Build on the CPU first:  python tools/probe/res_chain_variants.py build
usage on the GPU box: python tools/probe/res_chain_variants.py [iters] [taps]   (taps 1: encoder, 3: decoder)"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
# name -> EC_PROBE_FLAGS, or (EC_PROBE_FLAGS, extra -D defines)
VARIANTS = {"base": 0, "base2": 0, "no_gelu": 16, "scalar": (0, ["-DEC_SCALAR_GELU=1"]),
            "scalar_noslp": (0, ["-DEC_SCALAR_GELU=1", "-fno-slp-vectorize"]),
            "noslp": (0, ["-fno-slp-vectorize"])}


def build():
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    procs = []
    for name, fl in VARIANTS.items():
        fl, extra = fl if isinstance(fl, tuple) else (fl, [])
        out = os.path.join(HERE, "build", f"ec_{name}.so")
        procs.append(subprocess.Popen(
            ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wl,-Bsymbolic",
             f"-DEC_PROBE_FLAGS={fl}", *extra, "-I" + os.path.join(REPO, "include"), os.path.join(SRC, "reschain.hip"),
             os.path.join(SRC, "runtime.hip"), "-o", out]))
    for p in procs:
        assert p.wait() == 0


def main(iters=20, taps=1):
    import torch
    sys.path.insert(0, os.path.join(REPO, "vq-vae-transformer-arc-welding_amd"))
    from arcweld import _native as nat
    N, H, R, p = 16384, 512, 8, 0.1
    BF = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s, sc=1.0, dt=BF: (torch.randn(*s, device="cuda", generator=g) * sc).to(dt)  # noqa: E731
    e = lambda: torch.empty(N, H, device="cuda", dtype=BF)  # noqa: E731
    keep = []
    fa = nat.ResChainFwdArgs()
    fa.N, fa.H, fa.R, fa.drop_p, fa.taps, fa.seg = N, H, R, p, taps, 16
    a0, x0 = rnd(N, H), rnd(N, H)
    keep += [a0, x0]
    fa.a0, fa.x0 = a0.data_ptr(), x0.data_ptr()
    ctr = torch.ones(1, device="cuda", dtype=torch.int64)
    keep.append(ctr)
    fa.seed_ptr = ctr.data_ptr()
    fa.store_policy = 1
    ba = nat.ResChainBwdArgs()
    ba.N, ba.H, ba.R, ba.drop_p, ba.store_policy, ba.taps, ba.seg = N, H, R, p, 1, taps, 16
    TH = taps * H
    gx, gxo = rnd(N, H, sc=0.01), rnd(N, H, sc=0.01)
    keep += [gx, gxo]
    ba.gx, ba.gxo = gx.data_ptr(), gxo.data_ptr()
    for r in range(R):
        ts = [rnd(H, TH, sc=TH ** -0.5), rnd(H, TH, sc=TH ** -0.5), rnd(H, sc=0.1, dt=torch.float32),
              rnd(H, sc=0.1, dt=torch.float32), e(), e(), e(), e(), rnd(H, TH, sc=TH ** -0.5),
              rnd(H, TH, sc=TH ** -0.5), e(), e()]
        keep += ts
        fa.w1[r], fa.w2[r], fa.b1[r], fa.b2[r] = (t.data_ptr() for t in ts[:4])
        fa.h[r], fa.a1[r], fa.a[r] = ts[4].data_ptr(), ts[5].data_ptr(), ts[7].data_ptr()
        fa.x[r] = ts[6].data_ptr() if r < R - 1 else None
        fa.drop_seed[r] = r + 1
        ba.w1t[r], ba.w2t[r] = ts[8].data_ptr(), ts[9].data_ptr()
        ba.h[r], ba.x[r], ba.gh[r], ba.gxo_out[r] = ts[4].data_ptr(), ts[6].data_ptr(), ts[10].data_ptr(), \
            ts[11].data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    masks = torch.empty(R * (N // 64) * 512 * 8, device="cuda", dtype=torch.uint8)
    keep.append(masks)
    fa.drop_masks = ba.drop_masks = masks.data_ptr()
    pol = int(os.environ.get("EC_STORE_POLICY", "0"))
    fa.store_policy = ba.store_policy = pol
    print(f"taps {taps}, store policy {'WT (sc1)' if pol else 'NT'}")
    for name in VARIANTS:
        lib = ctypes.CDLL(os.path.join(HERE, "build", f"ec_{name}.so"))
        for fn in (lib.aw_res_chain_fwd, lib.aw_res_chain_bwd):
            fn.restype = ctypes.c_int
        sd = (ctypes.c_uint64 * R)(*range(1, R + 1))
        assert lib.aw_res_dropout_masks(ctypes.c_int64(N), R, ctypes.c_float(p), sd, ctypes.c_void_p(ctr.data_ptr()),
                                        ctypes.c_void_p(masks.data_ptr()), ctypes.c_void_p(s)) == 0
        res = []
        for fn, args in ((lib.aw_res_chain_fwd, fa), (lib.aw_res_chain_bwd, ba)):
            for _ in range(3):
                assert fn(ctypes.byref(args), ctypes.c_void_p(s)) == 0
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(iters):
                fn(ctypes.byref(args), ctypes.c_void_p(s))
            t1.record()
            torch.cuda.synchronize()
            res.append(t0.elapsed_time(t1) * 1000 / iters)
            if name.startswith("stamps"):
                import numpy as np
                buf = (ctypes.c_uint64 * (256 * 32 * 4))()
                lib.aw_probe_ec_stamps(buf, 256 * 32 * 4)
                st = np.frombuffer(buf, dtype=np.uint64).reshape(256, 32, 4).astype(np.int64)[:, :2 * R]
                loop = np.median(st[:, :, 1] - st[:, :, 0], axis=0)
                pub = np.median(st[:, :-1, 3] - st[:, :-1, 1], axis=0)
                epi = np.median(st[:, :-1, 2] - st[:, :-1, 3], axis=0)
                gap = np.median(st[:, 1:, 0] - st[:, :-1, 2], axis=0)
                print(f"  {'fwd' if args is fa else 'bwd'} stamps (cycles, median over WGs) k-loop {loop.astype(int).tolist()}")
                print(f"      k-loop end -> published {pub.astype(int).tolist()}")
                print(f"      published -> epilogue end {epi.astype(int).tolist()}")
                print(f"      -> next k-loop  {gap.astype(int).tolist()}")
        print(f"{name:14s} fwd {res[0]:7.1f} us   bwd {res[1]:7.1f} us", flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    else:
        main(*(int(v) for v in sys.argv[1:]))
