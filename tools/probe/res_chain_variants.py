"""Probe builds of csrc/reschain.hip: the chain kernels alone at the configs[1] shape with parts left out.  Each
variant is a copy of the product source with text replacements (the product carries no probe switches), compiled
with runtime.hip into tools/probe/build/ec_<name>.so.  Results of the probe builds are garbage by construction.
Build on the CPU first:  python tools/probe/res_chain_variants.py build
usage on the GPU box: python tools/probe/res_chain_variants.py [iters] [taps]   (taps 1: encoder, 3: decoder)"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(REPO, "vq-vae-transformer-arc-welding_amd", "csrc")
# name -> [(product text, replacement)]
VARIANTS = {
    "base": [],
    # every weight load reads the first 64 KB of its matrix (L1 / L2-resident)
    "l2weights": [("  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);\n  uint4 u;",
                   "  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff & 0xFFFF, 0);\n  uint4 u;")],
    # no global stores
    "nostore": [("  __builtin_amdgcn_raw_buffer_store_b128(u, r, voff, soff, WT ? 16 : 2);\n", "")],
    # the forward's GELU / GELU' replaced by the identity / one, the backward's GELU'(x_0) by one
    "nogelu": [("    const float phi = aw_phi_e(v[e], ex);", "    const float phi = 1.f;\n    ex = 0.f;"),
               ("for (int e = 0; e < 4; ++e) y[e] = gelu_erf_grad_fast(v[e]);", "for (int e = 0; e < 4; ++e) y[e] = 1.f;")],
}


def build():
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    src = open(os.path.join(SRC, "reschain.hip")).read()
    procs = []
    for name, reps in VARIANTS.items():
        text = src
        for a, b in reps:
            if text.count(a) != 1:
                sys.exit(f"{name}: text not found exactly once: {a[:60]!r}")
            text = text.replace(a, b)
        path = os.path.join(HERE, "build", f"ec_{name}.hip")
        open(path, "w").write(text)
        out = os.path.join(HERE, "build", f"ec_{name}.so")
        procs.append(subprocess.Popen(
            ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wl,-Bsymbolic",
             "-munsafe-fp-atomics", "-I" + SRC, "-I" + os.path.join(REPO, "include"), path,
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
    ba.gx, ba.gxo, ba.x0 = gx.data_ptr(), gxo.data_ptr(), x0.data_ptr()
    for r in range(R):
        ts = [rnd(H, TH, sc=TH ** -0.5), rnd(H, TH, sc=TH ** -0.5), rnd(H, sc=0.1, dt=torch.float32),
              rnd(H, sc=0.1, dt=torch.float32), e(), e(), e(), e(), rnd(H, TH, sc=TH ** -0.5),
              rnd(H, TH, sc=TH ** -0.5), e(), e()]
        keep += ts
        fa.w1[r], fa.w2[r], fa.b1[r], fa.b2[r] = (t.data_ptr() for t in ts[:4])
        fa.dgelu_h[r], fa.a1[r], fa.a[r] = ts[4].data_ptr(), ts[5].data_ptr(), ts[7].data_ptr()
        fa.dgelu_x[r] = ts[6].data_ptr() if r < R - 1 else None
        fa.drop_seed[r] = r + 1
        ba.w1t[r], ba.w2t[r] = ts[8].data_ptr(), ts[9].data_ptr()
        ba.dgelu_h[r], ba.dgelu_x[r], ba.gh[r], ba.gxo_out[r] = ts[4].data_ptr(), ts[6].data_ptr(), ts[10].data_ptr(), \
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
        print(f"{name:14s} fwd {res[0]:7.1f} us   bwd {res[1]:7.1f} us", flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["build"]:
        build()
    else:
        main(*(int(v) for v in sys.argv[1:]))
