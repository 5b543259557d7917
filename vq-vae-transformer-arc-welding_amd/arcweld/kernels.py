"""Typed wrappers over the C ABI (one function per entry point of include/arcweld_amd.h).

Every wrapper takes torch DEVICE tensors, derives sizes/leading dimensions from their strides, launches on the
current torch stream and raises on a non-zero status.  No wrapper has a CPU path.
"""
from __future__ import annotations

import contextvars
import ctypes

import torch

from . import _native as nat
from ._native import AW_ACT_DERIV, AW_ACT_GELU_ERF, AW_ACT_GELU_TANH, AW_BF16, AW_F32, GemmArgs, call, dtype_code, ptr, stream_ptr

__all__ = ["gemm", "AW_ACT_DERIV", "AW_ACT_GELU_ERF", "AW_ACT_GELU_TANH", "AW_BF16", "AW_F32"]


def _ld(t):
    if t is None:
        return 0
    if t.dim() == 1:
        return t.shape[0]
    if t.stride(-1) != 1:
        raise nat.NativeError("operand rows must be contiguous (stride(-1) == 1)")
    return t.stride(0)


# Epilogue store policy of the GEMMs issued inside a `store_policy(...)` block (aw_gemm_args.store_policy):
# nat.AW_STORE_NT (default) or nat.AW_STORE_WT (write-through: the VQ-VAE step, see arcweld/vqvae.py).
# The policy is context-local (a ContextVar): GEMMs issued from another thread, or from a callback that resets it
# (the VQ-VAE backward's mid_hook), keep their own.
_STORE_POLICY = contextvars.ContextVar("arcweld_store_policy", default=0)


class store_policy:
    """Context manager / decorator: GEMM launches issued inside use `policy` for their epilogue stores."""

    def __init__(self, policy):
        self.policy = int(policy)

    def __enter__(self):
        self._tok = _STORE_POLICY.set(self.policy)

    def __exit__(self, *exc):
        _STORE_POLICY.reset(self._tok)
        return False

    def __call__(self, fn):
        import functools

        @functools.wraps(fn)
        def wrapped(*a, **k):
            with store_policy(self.policy):
                return fn(*a, **k)
        return wrapped


# Optional live profiler: when set to a list, every gemm() appends (start_event, end_event, algorithmic_flops)
# recorded on the launch stream (bench.py uses it for the roofline of the GEMM kernel over the timed region).
PROFILE = None


def _algorithmic_flops(M, N, Kd, conv, flops):
    """2*M*N*K counting only taps that touch real input: the implicit k=3 conv loses one tap at each window
    edge (K_eff = cin*(3 - 2/seg)); callers with zero-padded operands (patch embed) pass `flops` explicitly."""
    if flops is not None:
        return float(flops)
    if conv is not None:
        seg = conv[1]
        return 2.0 * M * N * (Kd / 3.0) * (3.0 - 2.0 / seg)
    return 2.0 * M * N * Kd


def _gemm_args(A, B, M, N, K, *, a_trans=False, b_trans=False, conv=None, alpha=1.0, beta=0.0, bias=None,
               act=AW_ACT_GELU_ERF, pre=None, resid=None, drop=(0.0, 0), C=None, C2=None, c2_mode=0, drop2=(0.0, 0),
               colstats=None, stats_mod=0, a_rowsum=None, bias_mod=0, accumulate=False, col_map=(0, 1, 0),
               seed_ptr=None):
    if A.dtype != B.dtype:
        raise nat.NativeError(f"gemm operands must share a dtype ({A.dtype} vs {B.dtype})")
    a = GemmArgs()
    a.M, a.N, a.K = int(M), int(N), int(K)
    a.a_dtype = dtype_code(A.dtype)
    a.A, a.lda, a.a_trans = ptr(A), _ld(A), int(bool(a_trans))
    a.B, a.ldb, a.b_trans = ptr(B), _ld(B), int(bool(b_trans))
    if conv is not None:
        a.conv_cin, a.conv_seg, a.conv_dir, a.conv_operand = (int(v) for v in conv)
    a.alpha, a.beta = float(alpha), float(beta)
    a.bias = ptr(bias)
    a.act = int(act)
    a.store_policy = _STORE_POLICY.get()
    a.pre, a.ld_pre = ptr(pre), _ld(pre)
    if pre is not None:
        if pre.dtype not in (torch.float32, torch.bfloat16):
            raise nat.NativeError("pre must be float32 or bfloat16")
        a.pre_dtype = dtype_code(pre.dtype)
    a.resid, a.ld_resid = ptr(resid), _ld(resid)
    if resid is not None:
        if resid.dtype not in (torch.float32, torch.bfloat16):
            raise nat.NativeError("resid must be float32 or bfloat16")
        a.resid_dtype = dtype_code(resid.dtype)
    a.drop_p, a.drop_seed = float(drop[0]), int(drop[1]) & 0xFFFFFFFFFFFFFFFF
    if C is not None:
        a.C, a.ldc, a.c_dtype = ptr(C), _ld(C), dtype_code(C.dtype)
    if C2 is not None:
        a.C2, a.ldc2, a.c2_dtype = ptr(C2), _ld(C2), dtype_code(C2.dtype)
    a.c2_mode = int(c2_mode)
    a.drop2_p, a.drop2_seed = float(drop2[0]), int(drop2[1]) & 0xFFFFFFFFFFFFFFFF
    if colstats is not None:
        if colstats.dtype != torch.float64:
            raise nat.NativeError("colstats must be float64")
        a.colstats, a.stats_mod = ptr(colstats), int(stats_mod)
    a.a_rowsum = ptr(a_rowsum)
    a.bias_mod = int(bias_mod)
    a.accumulate = int(bool(accumulate))
    a.col_mod, a.col_mul, a.col_off = (int(v) for v in col_map)
    a.seed_ptr = ptr(seed_ptr)
    return a


def _timed(s, fn, flops, tag, name=None, nbytes=None):
    """Bench profiling (PROFILE is a list): HIP events around one launch on its stream, with the launch's
    algorithmic FLOPs, a kernel-family tag ("gemm_bf16", "gemm_f32", "attn_fwd", "attn_bwd", "vq_fwd"), the name of
    the kernel it runs (the rocprofv3 kernel name's stem, for the per-kernel roofline) and its algorithmic HBM bytes
    (None where not stated)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    fn(s.cuda_stream)
    e1.record(s)
    PROFILE.append((e0, e1, flops, tag, name or tag, nbytes))


def _gemm_tag(A):
    return "gemm_bf16" if A.dtype == torch.bfloat16 else "gemm_f32"


def gemm(A, B, M, N, K, *, stream=None, flops=None, **kw):
    """C = epilogue(alpha * op(A) @ op(B)); see aw_gemm in include/arcweld_amd.h for the exact semantics.

    conv = (cin, seg, dir, operand) selects the implicit k=3 convolution form."""
    a = _gemm_args(A, B, M, N, K, **kw)
    lib = nat.load()
    wsn = lib.aw_gemm_workspace(ctypes.byref(a))
    ws = torch.empty(wsn, device=A.device, dtype=torch.float32) if wsn > 0 else None
    if PROFILE is None:
        call("aw_gemm_ws", ctypes.byref(a), ptr(ws), wsn, stream_ptr(stream))
        return kw.get("C")
    s = stream if stream is not None else torch.cuda.current_stream()
    _timed(s, lambda sp: call("aw_gemm_ws", ctypes.byref(a), ptr(ws), wsn, sp),
           _algorithmic_flops(M, N, K, kw.get("conv"), flops), _gemm_tag(A), "gemm_kernel")
    return kw.get("C")


MAX_GROUPS = 16


def gemm_grouped(problems, stream=None):
    """One aw_gemm_grouped launch per chunk of <= 16 accumulate-mode problems that share everything except
    (A, B, C, a_rowsum).  ``problems`` is a list of (A, B, M, N, K, kwargs) tuples as for ``gemm``."""
    for c0 in range(0, len(problems), MAX_GROUPS):
        chunk = problems[c0:c0 + MAX_GROUPS]
        arr = (GemmArgs * len(chunk))(*[_gemm_args(A, B, M, N, K, **kw) for (A, B, M, N, K, kw) in chunk])
        if PROFILE is None:
            call("aw_gemm_grouped", arr, len(chunk), stream_ptr(stream))
            continue
        s = stream if stream is not None else torch.cuda.current_stream()
        fl = sum(_algorithmic_flops(M, N, K, kw.get("conv"), None) for (_, _, M, N, K, kw) in chunk)
        c0_ = chunk[0]
        # the grouped decoder k = 3 weight gradients run wgrad_conv3_kernel (csrc/wgrad.hip wgrad_conv3_try)
        nm = "wgrad_conv3_kernel" if (c0_[5].get("conv") is not None and c0_[0].dtype == torch.bfloat16) \
            else "gemm_kernel (grouped)"
        _timed(s, lambda sp: call("aw_gemm_grouped", arr, len(chunk), sp), fl, _gemm_tag(chunk[0][0]), nm)


WGRAD_BATCH_MAX = 32     # aw_wgrad_batch problems per launch (include/arcweld_amd.h AW_WGRAD_BATCH_MAX)


def wgrad_batch_ok(problems):
    """True when aw_wgrad_batch takes these problems (bf16 operands, M / N multiples of 256, one K) and pays: at least
    128 of its 256 x 256 tiles (the transformer's half-step batch of four Linear kinds, 192 tiles: 656 -> 532 us per
    launch in tools/probe/wgrad_tt_probe.py, the decoder step 5.58 -> 5.44 ms same box).  Below that its split-K
    fix-up costs more than it saves (the VQ-VAE encoder's 64 tiles: 214 vs 184 us for the grouped launch), and the
    per-shape grouped launches run instead.  ARCWELD_WGRAD_BATCH=0 / 1 forces them off / on (A/B, tests)."""
    import os
    mode = os.environ.get("ARCWELD_WGRAD_BATCH", "auto")
    if mode == "0" or not problems or len(problems) > WGRAD_BATCH_MAX:
        return False
    arr = (GemmArgs * len(problems))(*[_gemm_args(A, B, M, N, K, **kw) for (A, B, M, N, K, kw) in problems])
    if nat.load().aw_wgrad_batch_workspace(arr, len(problems)) <= 0:
        return False
    tiles = sum((M // 256) * (N // 256) for (_, _, M, N, _, _) in problems)
    return mode == "1" or tiles >= 128


def wgrad_batch(problems, stream=None):
    """One aw_wgrad_batch launch over <= 32 weight-gradient problems (A, B, M, N, K, kwargs) as for ``gemm`` (M and
    N may differ between problems; K, alpha and the dtype may not); the stream-K workspace comes from the caching
    allocator."""
    arr = (GemmArgs * len(problems))(*[_gemm_args(A, B, M, N, K, **kw) for (A, B, M, N, K, kw) in problems])
    lib = nat.load()
    wsb = lib.aw_wgrad_batch_workspace(arr, len(problems))
    if wsb < 0:
        raise nat.NativeError(f"aw_wgrad_batch: batch not eligible ({lib.aw_last_error().decode(errors='replace')})")
    ws = torch.empty((wsb + 3) // 4, device=problems[0][0].device, dtype=torch.float32)
    if PROFILE is None:
        call("aw_wgrad_batch", arr, len(problems), ptr(ws), wsb, stream_ptr(stream))
        return
    s = stream if stream is not None else torch.cuda.current_stream()
    fl = sum(_algorithmic_flops(M, N, K, None, None) for (_, _, M, N, K, _) in problems)
    _timed(s, lambda sp: call("aw_wgrad_batch", arr, len(problems), ptr(ws), wsb, sp), fl, _gemm_tag(problems[0][0]),
           "wgrad_tt_kernel")


def wgrad_issue(problems, stream=None):
    """Weight-gradient problems of one backward region that share K: in aw_wgrad_batch launches of <= 32 problems
    when eligible (bf16, M / N multiples of 256), else one aw_gemm_grouped launch per shape."""
    if not problems:
        return
    nch = (len(problems) + WGRAD_BATCH_MAX - 1) // WGRAD_BATCH_MAX
    per = (len(problems) + nch - 1) // nch
    chunks = [problems[i:i + per] for i in range(0, len(problems), per)]
    if all(wgrad_batch_ok(c) for c in chunks):
        for c in chunks:
            wgrad_batch(c, stream)
        return
    by_shape = {}
    for pb in problems:
        by_shape.setdefault((pb[2], pb[3]), []).append(pb)
    for grp in by_shape.values():
        gemm_grouped(grp, stream)


# ------------------------------------------------------------------------------------------------ encoder chain
RES_CHAIN_MAX = nat.RES_CHAIN_MAX


def res_chain_ok(H, R, T, RT, taps=1, seg=16, which="ENC"):
    """aw_res_chain_fwd / _bwd serve the bf16 operand mode with bf16 residual streams, H == 512 and 1 <= R <= 16
    (ResBlocks without BatchNorm): the encoder's per-token stack (taps 1) and the decoder's k = 3 stack over 16-token
    windows (taps 3, seg 16).  ARCWELD_ENC_CHAIN=0 / ARCWELD_DEC_CHAIN=0 keep the per-conv GEMM launches of that
    stack (A/B runs, and the tests that compare the two)."""
    import os
    if os.environ.get(f"ARCWELD_{which}_CHAIN", "1") == "0":
        return False
    return (H == 512 and 1 <= R <= RES_CHAIN_MAX and T == torch.bfloat16 and RT == torch.bfloat16
            and (taps == 1 or (taps == 3 and seg == 16)))


def _chain_store_policy():
    """The chain's store policy: non-temporal (ARCWELD_CHAIN_STORE=wt: write-through, for A/B runs).  Same-box
    A/B of the VQ-VAE step: 2.932 / 2.914 ms nt vs 2.971 / 2.959 ms wt (the GEMM launches it replaces use wt)."""
    import os
    return nat.AW_STORE_WT if os.environ.get("ARCWELD_CHAIN_STORE", "nt") == "wt" else nat.AW_STORE_NT


def _chk_rows(ts, N, H, who):
    for t in ts:
        if t is None:
            continue
        if t.dtype != torch.bfloat16 or t.dim() != 2 or tuple(t.shape) != (N, H) or not t.is_contiguous():
            raise nat.NativeError(f"{who}: activations must be contiguous ({N}, {H}) bfloat16 tensors")


def res_dropout_masks_empty(N, R, device):
    """An uninitialised buffer for the chain's dropout keep bits of R blocks at N tokens (res_chain_fwd fills it)."""
    nb = nat.load().aw_res_dropout_masks_bytes(int(N), int(R))
    if nb <= 0:
        raise nat.NativeError("res_dropout_masks: bad N / R")
    return torch.empty(nb, device=device, dtype=torch.uint8)


def res_dropout_masks(N, drop, seed_ptr=None, stream=None):
    """The chain's dropout keep bits for drop = (p, R seeds) at N tokens (aw_res_dropout_masks, the standalone form of
    what res_chain_fwd writes): a uint8 device tensor, or None when p == 0."""
    p, seeds = float(drop[0]), list(drop[1] or [])
    if p <= 0.0:
        return None
    R = len(seeds)
    out = res_dropout_masks_empty(N, R, torch.cuda.current_device() if seed_ptr is None else seed_ptr.device)
    sd = (ctypes.c_uint64 * R)(*[int(v) & 0xFFFFFFFFFFFFFFFF for v in seeds])
    call("aw_res_dropout_masks", int(N), R, p, sd, ptr(seed_ptr), ptr(out), stream_ptr(stream))
    return out


def _nbytes(ts):
    """Algorithmic HBM bytes of a launch: every operand read once and every output written once (distinct tensors;
    None entries are absent operands)."""
    seen, n = set(), 0
    for t in ts:
        if t is not None and t.data_ptr() not in seen:
            seen.add(t.data_ptr())
            n += t.numel() * t.element_size()
    return n


def _chain_flops(R, N, H, taps, seg):
    """Algorithmic flops of one chain launch: 2R convs of 2 N H (taps H) -- for taps 3 only the taps that touch a
    real row (the window edges lose one tap each, as _algorithmic_flops counts the implicit conv GEMMs)."""
    if taps == 1:
        return 4.0 * R * N * H * H
    return 4.0 * R * N * H * H * (3 - 2.0 / seg)


def res_chain_fwd(a0, x0, w1, w2, b1, b2, dh, a1, dx, a, drop=(0.0, None), seed_ptr=None, masks=None, taps=1, seg=16,
                  stream=None):
    """One aw_res_chain_fwd launch over the R = len(w1) ResBlocks (see include/arcweld_amd.h).

    a0 / x0: (N, H) bf16; w1 / w2: R packed weight copies (res_pack_weights); b1 / b2: R f32 biases; dh / a1 / dx / a:
    R output tensors each -- dh[r] = GELU'(h_r), a1[r], dx[r] = GELU'(x_{r+1}) (the backward's multipliers), a[r]
    (dh, a1, dx entries may be None: not stored; dx[R-1] is never stored); drop = (p, R seeds); masks: None or a
    res_dropout_masks_empty(N, R) buffer the launch fills with the keep bits (for res_chain_bwd)."""
    N, H = a0.shape
    R = len(w1)
    if not (1 <= R <= RES_CHAIN_MAX) or not all(len(v) == R for v in (w2, b1, b2, dh, a1, dx, a)):
        raise nat.NativeError("res_chain_fwd: need R (1..16) entries in every per-block list")
    _chk_rows([a0, x0] + list(dh) + list(a1) + list(dx) + list(a), N, H, "res_chain_fwd")
    g = nat.ResChainFwdArgs()
    g.N, g.H, g.R, g.taps, g.seg = N, H, R, int(taps), int(seg)
    g.a0, g.x0 = ptr(a0), ptr(x0)
    for r in range(R):
        g.w1[r], g.w2[r], g.b1[r], g.b2[r] = ptr(w1[r]), ptr(w2[r]), ptr(b1[r]), ptr(b2[r])
        g.dgelu_h[r], g.a1[r], g.dgelu_x[r], g.a[r] = ptr(dh[r]), ptr(a1[r]), ptr(dx[r]), ptr(a[r])
        g.drop_seed[r] = int(drop[1][r]) & 0xFFFFFFFFFFFFFFFF if drop[0] > 0 else 0
    g.drop_p = float(drop[0])
    g.seed_ptr = ptr(seed_ptr)
    g.store_policy = _chain_store_policy()
    g.drop_masks = ptr(masks)
    _maybe_timed(stream, "gemm_bf16", _chain_flops(R, N, H, taps, seg),
                 lambda sp: call("aw_res_chain_fwd", ctypes.byref(g), sp), f"res_chain_fwd_kernel<{int(taps)}>",
                 _nbytes([a0, x0, masks] + list(w1) + list(w2) + list(b1) + list(b2) + list(dh) + list(a1) +
                         list(dx)[:-1] + list(a)))


def res_chain_bwd(gx, gxo, w1t, w2t, dh, x0, dx, gh, gxo_out, drop_p=0.0, masks=None, taps=1, seg=16, stream=None):
    """One aw_res_chain_bwd launch (see include/arcweld_amd.h): w1t / w2t are the packed backward copies, dh the
    forward's saved GELU'(h_r), x0 the stack input x_0 and dx[r] (r >= 1) the forward's GELU'(x_r) (dx[0] is not read:
    GELU'(x_0) is evaluated in the launch), gh / gxo_out the R outputs each; masks (drop_p > 0, R > 1): the keep bits
    res_chain_fwd wrote (or res_dropout_masks made)."""
    N, H = gx.shape
    R = len(w1t)
    if not (1 <= R <= RES_CHAIN_MAX) or not all(len(v) == R for v in (w2t, dh, dx, gh, gxo_out)):
        raise nat.NativeError("res_chain_bwd: need R (1..16) entries in every per-block list")
    _chk_rows([gx, gxo, x0] + list(dh) + list(dx[1:]) + list(gh) + list(gxo_out), N, H, "res_chain_bwd")
    g = nat.ResChainBwdArgs()
    g.N, g.H, g.R, g.taps, g.seg = N, H, R, int(taps), int(seg)
    g.gx, g.gxo, g.x0 = ptr(gx), ptr(gxo), ptr(x0)
    for r in range(R):
        g.w1t[r], g.w2t[r], g.dgelu_h[r] = ptr(w1t[r]), ptr(w2t[r]), ptr(dh[r])
        g.dgelu_x[r] = ptr(dx[r]) if r > 0 else None
        g.gh[r], g.gxo_out[r] = ptr(gh[r]), ptr(gxo_out[r])
    g.drop_p = float(drop_p)
    g.store_policy = _chain_store_policy()
    g.drop_masks = ptr(masks)
    _maybe_timed(stream, "gemm_bf16", _chain_flops(R, N, H, taps, seg),
                 lambda sp: call("aw_res_chain_bwd", ctypes.byref(g), sp), f"res_chain_bwd_kernel<{int(taps)}>",
                 _nbytes([gx, gxo, x0, masks] + list(w1t) + list(w2t) + list(dh) + list(dx[1:]) + list(gh) +
                         list(gxo_out)))


def res_pack_weights(src, fwd=None, bwd=None, taps=1, stream=None):
    """Fragment-packed copies of [512][taps*512] bf16 [out][(tap, in)] weights for the chain (aw_res_pack_weights):
    fwd[i] <- W packed (aw_res_chain_fwd's w1 / w2), bwd[i] <- the backward operand packed (aw_res_chain_bwd's w1t /
    w2t); either list may be None.  One launch per 32 matrices."""
    n = len(src)
    fwd = fwd if fwd is not None else [None] * n
    bwd = bwd if bwd is not None else [None] * n
    if len(fwd) != n or len(bwd) != n:
        raise nat.NativeError("res_pack_weights: list lengths differ")
    for t in list(src) + [t for t in fwd + bwd if t is not None]:
        if t.dtype != torch.bfloat16 or t.numel() != 512 * 512 * taps or not t.is_contiguous():
            raise nat.NativeError(f"res_pack_weights: need contiguous 512 x {512 * taps} bfloat16 tensors")
    for c0 in range(0, n, nat.RES_PACK_MAX):
        sl = slice(c0, c0 + nat.RES_PACK_MAX)
        m = len(src[sl])
        arr = lambda ts: (ctypes.c_void_p * m)(*[ptr(t) for t in ts])  # noqa: E731
        call("aw_res_pack_weights", arr(src[sl]), arr(fwd[sl]), arr(bwd[sl]), m, int(taps), stream_ptr(stream))


# ------------------------------------------------------------------------------------------------ VQ
def vq_forward(z2d, E, zq, idx, counts, sqerr, stream=None, zq_copy=None, count_groups=1):
    """zq_copy: optional bf16/f32 tensor that also receives z_q.  count_groups > 1: counts holds that many partial
    histograms of K floats (aw_vq_forward_ex2; vq_finalize sums them)."""
    N, D = z2d.shape
    Kc = E.shape[0]
    assert counts.numel() >= count_groups * Kc, "counts: count_groups x K floats"
    # the pinned kernel (codebook in LDS, f32-input MFMA) serves K <= 512, D in {16, 32, 64} (csrc/vq.hip)
    name = "vq_fwd_pinned_kernel" if Kc <= 512 and D in (16, 32, 64) else "vq_fwd_kernel"
    _maybe_timed(stream, "vq_fwd", 2.0 * N * Kc * D, lambda sp: call(
        "aw_vq_forward_ex2", ptr(z2d), ptr(E), N, Kc, D, ptr(zq), ptr(idx), ptr(counts), int(count_groups),
        ptr(sqerr), ptr(zq_copy), dtype_code(zq_copy.dtype) if zq_copy is not None else 0, sp), name,
        _nbytes([z2d, E, zq, idx, zq_copy]) + 4 * Kc * count_groups)


def vq_finalize(counts, sqerr, N, K, D, beta, loss, perplexity, stream=None, count_groups=1):
    call("aw_vq_finalize_ex", ptr(counts), int(count_groups), ptr(sqerr), N, K, D, float(beta), ptr(loss),
         ptr(perplexity), stream_ptr(stream))


def vq_backward(z2d, E, idx, g_zq, g_loss, beta, dz, dE, stream=None, dz_copy=None):
    """dz_copy: optional bf16/f32 tensor that also receives dz (aw_vq_backward_ex)."""
    N, D = z2d.shape
    if dz_copy is None:
        call("aw_vq_backward", ptr(z2d), ptr(E), ptr(idx), ptr(g_zq), ptr(g_loss), N, E.shape[0], D, float(beta),
             ptr(dz), ptr(dE), stream_ptr(stream))
    else:
        call("aw_vq_backward_ex", ptr(z2d), ptr(E), ptr(idx), ptr(g_zq), ptr(g_loss), N, E.shape[0], D, float(beta),
             ptr(dz), ptr(dE), ptr(dz_copy), dtype_code(dz_copy.dtype), stream_ptr(stream))


# ------------------------------------------------------------------------ residual VQ (EMA codebooks)
def vq_cluster_sums(z2d, idx, K, sums, stream=None):
    """sums[idx[n]] += z[n] (sums zeroed by the caller)."""
    _dense(z2d, "vq_cluster_sums")
    call("aw_vq_cluster_sums", ptr(z2d), ptr(idx), z2d.shape[0], K, z2d.shape[1], ptr(sums), stream_ptr(stream))


def kmeans_update(means, sums, counts, avg=None, stream=None):
    call("aw_kmeans_update", ptr(means), ptr(sums), ptr(counts), means.shape[0], means.shape[1], ptr(avg),
         stream_ptr(stream))


def rvq_ema_update(embed, embed_avg, cluster_size, counts, sums, z2d, decay, eps, threshold, salt, seed_ptr, ws,
                   stream=None):
    K, D = embed.shape
    call("aw_rvq_ema_update", ptr(embed), ptr(embed_avg), ptr(cluster_size), ptr(counts), ptr(sums), ptr(z2d),
         z2d.shape[0], K, D, float(decay), float(eps), float(threshold), int(salt) & 0xFFFFFFFFFFFFFFFF,
         ptr(seed_ptr), ptr(ws), stream_ptr(stream))


def rvq_residual(r, zq, out, first, r_next=None, stream=None):
    call("aw_rvq_residual", ptr(r), ptr(zq), zq.numel(), ptr(out), int(bool(first)), ptr(r_next), stream_ptr(stream))


def rvq_backward(res, q, g_zq, g_loss, dz, commitment=1.0, stream=None):
    """res, q: (nq, N, D); dz (N, D)."""
    nq, N, D = res.shape
    call("aw_rvq_backward", ptr(res), ptr(q), ptr(g_zq), ptr(g_loss), nq, N, D, float(commitment), ptr(dz),
         stream_ptr(stream))


def vq_onehot(idx, K, out, stream=None):
    call("aw_vq_onehot", ptr(idx), idx.numel(), K, ptr(out), stream_ptr(stream))


def vq_gather(E, idx, out, stream=None):
    call("aw_vq_gather", ptr(E), ptr(idx), idx.numel(), E.shape[1], ptr(out), stream_ptr(stream))


# ------------------------------------------------------------------------------------------ layouts
def patchify(x, P, out, stream=None):
    B, L, C = x.shape
    call("aw_patchify", ptr(x), B, L, C, P, ptr(out), out.stride(0), dtype_code(out.dtype), stream_ptr(stream))


def weight_relayout(W, O, I, k, tap, mode, out, ldo=0, stream=None):
    _dense(W, "weight_relayout")
    call("aw_weight_relayout", ptr(W), O, I, k, tap, mode, ptr(out), ldo, dtype_code(out.dtype), stream_ptr(stream))


RELAYOUT_MAX_JOBS = 40


def _dense(W, who):
    if not W.is_contiguous():
        raise nat.NativeError(f"{who}: the source weight must be contiguous (got strides {tuple(W.stride())})")


def weight_relayout_batch(jobs, stream=None):
    """Many weight_relayout calls in one launch per output dtype.  jobs: (W, O, I, k, tap, mode, out[, ldo]);
    mode 5 is a plain cast of O*I elements."""
    by_dtype = {}
    for jb in jobs:
        by_dtype.setdefault(jb[6].dtype, []).append(jb)
    for dt, js in by_dtype.items():
        for c0 in range(0, len(js), RELAYOUT_MAX_JOBS):
            chunk = js[c0:c0 + RELAYOUT_MAX_JOBS]
            arr = (nat.RelayoutJob * len(chunk))()
            for r, jb in zip(arr, chunk):
                W, O, I, k, tap, mode, out = jb[:7]
                _dense(W, "weight_relayout_batch")
                r.W, r.out = ptr(W), ptr(out)
                r.O, r.I, r.k, r.tap, r.mode = int(O), int(I), int(k), int(tap), int(mode)
                r.ldo = int(jb[7]) if len(jb) > 7 else 0
            call("aw_weight_relayout_batch", arr, len(chunk), dtype_code(dt), stream_ptr(stream))


def weight_grad_scatter(g, O, I, k, tap, mode, G, stream=None):
    call("aw_weight_grad_scatter", ptr(g), O, I, k, tap, mode, g.stride(0), ptr(G), stream_ptr(stream))


def cast(x, out, stream=None):
    call("aw_cast", ptr(x), x.numel(), ptr(out), dtype_code(out.dtype), stream_ptr(stream))


def bn_finalize(colstats, n, H, gamma, beta, rm, rv, nbt, eps, momentum, training, stats, stream=None):
    call("aw_bn_finalize", ptr(colstats), n, H, ptr(gamma), ptr(beta), ptr(rm), ptr(rv), ptr(nbt), float(eps),
         float(momentum), int(training), ptr(stats), stream_ptr(stream))


def unpatch_head_fwd(y, Q, stats, w2, b2, x_hat, stream=None):
    """y (R, H) f32 or bf16 (the ConvT output in the bf16 operand mode)."""
    R, H = y.shape
    call("aw_unpatch_head_fwd_ex", ptr(y), dtype_code(y.dtype), R, H, Q, ptr(stats), ptr(w2), ptr(b2), ptr(x_hat),
         stream_ptr(stream))


def unpatch_head_bwd1(y, Q, stats, w2, g_xhat, gsums, gw2, gb2, ggamma, gbeta, stream=None):
    R, H = y.shape
    call("aw_unpatch_head_bwd1_ex", ptr(y), dtype_code(y.dtype), R, H, Q, ptr(stats), ptr(w2), ptr(g_xhat), ptr(gsums),
         ptr(gw2), ptr(gb2), ptr(ggamma), ptr(gbeta), stream_ptr(stream))


def unpatch_head_bwd2(y, Q, stats, w2, g_xhat, gsums, training, g_y, db_y, stream=None):
    R, H = y.shape
    call("aw_unpatch_head_bwd2_ex", ptr(y), dtype_code(y.dtype), R, H, Q, ptr(stats), ptr(w2), ptr(g_xhat),
         ptr(gsums), int(training), ptr(g_y), dtype_code(g_y.dtype), ptr(db_y), stream_ptr(stream))


def unpatch_head_fwd_bwd1(y, Q, stats, w2, b2, x, gscale, x_hat, g_xhat, sqerr, gsums, gw2, gb2, ggamma, gbeta,
                          stream=None):
    """Fused training-step head: forward + MSE value / gradient + backward pass 1 in one read of y (H == 512).
    The kernel reads x, x_hat and g_xhat as R*5 contiguous f32 values (its buffer range check would silently
    return zeros for a shorter x), so their sizes are checked here."""
    R, H = y.shape
    for nm, t in (("x", x), ("x_hat", x_hat), ("g_xhat", g_xhat)):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != R * 5:
            raise nat.NativeError(f"unpatch_head_fwd_bwd1: {nm} must be a contiguous float32 tensor of R*5 = {R * 5} "
                                  f"elements (got {tuple(t.shape)} {t.dtype}, contiguous={t.is_contiguous()})")
    call("aw_unpatch_head_fwd_bwd1", ptr(y), dtype_code(y.dtype), R, H, Q, ptr(stats), ptr(w2), ptr(b2), ptr(x),
         ptr(gscale), ptr(x_hat), ptr(g_xhat), ptr(sqerr), ptr(gsums), ptr(gw2), ptr(gb2), ptr(ggamma), ptr(gbeta),
         stream_ptr(stream))


def head_bf16_ok(H):
    """The head passes take a bf16 ConvT output when H is a power of two in 64..2048 (aw_unpatch_head_*_ex)."""
    return 64 <= H <= 2048 and H & (H - 1) == 0


def mse_fwd(a, b, sqerr, stream=None):
    call("aw_mse_fwd", ptr(a), ptr(b), a.numel(), ptr(sqerr), stream_ptr(stream))


def mse_bwd(a, b, g, ga, stream=None):
    call("aw_mse_bwd", ptr(a), ptr(b), a.numel(), ptr(g), ptr(ga), stream_ptr(stream))


def scalar_add(a, b, out, stream=None):
    call("aw_scalar_add", ptr(a), ptr(b), ptr(out), stream_ptr(stream))


def mse_finalize(sqerr, numel, out, stream=None):
    call("aw_mse_finalize", ptr(sqerr), int(numel), ptr(out), stream_ptr(stream))


def mse_finalize_add(sqerr, numel, addend, out, total, stream=None):
    """out = sqerr / numel and total = out + addend (device scalars), in one launch."""
    call("aw_mse_finalize_add", ptr(sqerr), int(numel), ptr(addend), ptr(out), ptr(total), stream_ptr(stream))


# ------------------------------------------------------------------------------------------ optimizer
def radam_step(param, grad, m, v, seg_off, seg_len, seg_wd, seg_active, nseg, total, step, lr, beta1, beta2, eps,
               gscale=None, stream=None, step_ptr=None, ops=None, zero_grad=False):
    """aw_radam_step, or aw_radam_step_ops when `ops` (device table of aw_operand_desc, AW_OPS_PER_SEG per
    segment) is given: the update also writes the operand copies of the updated weights.  zero_grad: the updated
    elements' gradients are zeroed in the same pass."""
    args = (ptr(param), ptr(grad), ptr(m), ptr(v), ptr(seg_off), ptr(seg_len), ptr(seg_wd), ptr(seg_active), int(nseg),
            int(total), int(step), float(lr), float(beta1), float(beta2), float(eps), ptr(gscale), ptr(step_ptr))
    if ops is None:
        call("aw_radam_step", *args, int(bool(zero_grad)), stream_ptr(stream))
    else:
        call("aw_radam_step_ops", *args, ptr(ops), int(bool(zero_grad)), stream_ptr(stream))


def counter_add_snapshot(counter, snapshot, v=1, stream=None, zero=None):
    """counter += v and snapshot = the new value, in one launch; `zero` (a contiguous float64 tensor) is zeroed by
    the same launch."""
    if zero is None:
        call("aw_counter_add_snapshot", ptr(counter), int(v), ptr(snapshot), stream_ptr(stream))
        return
    if zero.dtype != torch.float64 or not zero.is_contiguous():
        raise nat.NativeError("counter_add_snapshot: zero must be a contiguous float64 tensor")
    call("aw_counter_add_snapshot_zero", ptr(counter), int(v), ptr(snapshot), ptr(zero), zero.numel(),
         stream_ptr(stream))


def counter_add(counter, v=1, stream=None):
    """counter (int64 device tensor) += v on the stream (per-step RNG / optimizer-step counters)."""
    call("aw_counter_add", ptr(counter), int(v), stream_ptr(stream))


NORM_WS = 1024      # AW_NORM_WS


def grad_norm_clip(grad, seg_off, seg_len, seg_active, nseg, max_norm, ws, out_norm, out_coef, stream=None):
    if ws.numel() < NORM_WS or ws.dtype != torch.float64:
        raise nat.NativeError(f"grad_norm_clip: ws must hold {NORM_WS} float64")
    call("aw_grad_norm_clip", ptr(grad), ptr(seg_off), ptr(seg_len), ptr(seg_active), int(nseg), grad.numel(),
         float(max_norm), ptr(ws), ptr(out_norm), ptr(out_coef), stream_ptr(stream))


def scale_(x, s, stream=None):
    call("aw_scale", ptr(x), x.numel(), ptr(s), stream_ptr(stream))


# ---------------------------------------------------------------------------------------- transformer
def layernorm_fwd(x, w, b, eps, y, mean, rstd, stream=None):
    R, D = x.shape
    call("aw_layernorm_fwd", ptr(x), R, D, ptr(w), ptr(b), float(eps), ptr(y), dtype_code(y.dtype), ptr(mean),
         ptr(rstd), stream_ptr(stream))


def layernorm_bwd(x, dy, w, mean, rstd, dx, accumulate, dw, db, dx2=None, drop=(0.0, 0), stream=None,
                  seed_ptr=None):
    R, D = x.shape
    call("aw_layernorm_bwd", ptr(x), ptr(dy), R, D, ptr(w), ptr(mean), ptr(rstd), ptr(dx), int(accumulate), ptr(dw),
         ptr(db), ptr(dx2), dtype_code(dx2.dtype) if dx2 is not None else AW_F32, float(drop[0]),
         int(drop[1]) & 0xFFFFFFFFFFFFFFFF, ptr(seed_ptr), stream_ptr(stream))


def class_head_fwd(xf, B, T, w1, b1, W2, b2, s, out, stream=None):
    call("aw_class_head_fwd", ptr(xf), B, T, xf.shape[-1], ptr(w1), ptr(b1), ptr(W2), ptr(b2), ptr(s), ptr(out),
         stream_ptr(stream))


def class_head_bwd(xf, s, dout, B, T, w1, W2, dxf, dw1, db1, dW2, db2, stream=None):
    call("aw_class_head_bwd", ptr(xf), ptr(s), ptr(dout), B, T, xf.shape[-1], ptr(w1), ptr(W2), ptr(dxf), ptr(dw1),
         ptr(db1), ptr(dW2), ptr(db2), stream_ptr(stream))


def embed_fwd(ids, wtok, pe, x, stream=None):
    B, T = ids.shape
    call("aw_embed_fwd", ptr(ids), B, T, wtok.shape[1], ptr(wtok), ptr(pe), ptr(x), stream_ptr(stream))


def embed_ln_fwd(ids, wtok, pe, x, w, b, eps, y, mean, rstd, stream=None):
    """embed_fwd followed by layernorm_fwd(x, ...) in one launch (d_model 256/512/768/1024), bit-identical to the pair."""
    B, T = ids.shape
    call("aw_embed_ln_fwd", ptr(ids), B, T, wtok.shape[1], ptr(wtok), ptr(pe), ptr(x), ptr(w), ptr(b), float(eps),
         ptr(y), dtype_code(y.dtype), ptr(mean), ptr(rstd), stream_ptr(stream))


def embed_bwd(ids, dx, dwtok, stream=None, sort=True):
    """dwtok[ids[r]] += dx[r].  sort: the counting-sort form (aw_embed_bwd_sorted; scratch allocated here), else the
    atomic form."""
    B, T = ids.shape
    if not sort:
        call("aw_embed_bwd", ptr(ids), B, T, dwtok.shape[1], ptr(dx), ptr(dwtok), stream_ptr(stream))
        return
    V = dwtok.shape[0]
    work = torch.empty(V + 1 + B * T, device=dx.device, dtype=torch.int32)
    call("aw_embed_bwd_sorted", ptr(ids), B, T, dwtok.shape[1], V, ptr(dx), ptr(dwtok), ptr(work),
         stream_ptr(stream))


EMBED_SORT_MAX_V = 15360


def embed_sort(ids, V, work, stream=None):
    """The counting sort half of embed_bwd (work: V + 1 + ids.numel() int32)."""
    call("aw_embed_sort", ptr(ids), ids.numel(), V, ptr(work), stream_ptr(stream))


def embed_bwd_segsum(work, dx, dwtok, stream=None):
    """The table-row sums half of embed_bwd, from embed_sort's work."""
    call("aw_embed_bwd_segsum", ptr(work), dwtok.shape[0], dwtok.shape[1], ptr(dx), ptr(dwtok), stream_ptr(stream))


def attn_flops(B, T, n_head, d):
    """Algorithmic FLOPs of the causal attention forward: QK^T and PV over the T(T+1)/2 causal pairs per head."""
    return 4.0 * B * n_head * (T * (T + 1) / 2) * (d // n_head)


def _maybe_timed(stream, tag, flops, fn, name=None, nbytes=None):
    if PROFILE is None:
        fn(stream_ptr(stream))
        return
    s = stream if stream is not None else torch.cuda.current_stream()
    _timed(s, fn, flops, tag, name, nbytes)


def attn_fwd(qkv, B, T, n_head, d, y, lse, drop=(0.0, 0), seed_ptr=None, stream=None):
    """drop = (p, seed): attention-probability dropout (aw_attn_fwd_dropout); p = 0 is plain aw_attn_fwd."""
    if drop[0] > 0:
        _maybe_timed(stream, "attn_fwd", attn_flops(B, T, n_head, d), lambda sp: call(
            "aw_attn_fwd_dropout", ptr(qkv), B, T, n_head, d, dtype_code(qkv.dtype), ptr(y), ptr(lse),
            float(drop[0]), int(drop[1]) & 0xFFFFFFFFFFFFFFFF, ptr(seed_ptr), sp))
        return
    _maybe_timed(stream, "attn_fwd", attn_flops(B, T, n_head, d), lambda sp: call(
        "aw_attn_fwd", ptr(qkv), B, T, n_head, d, dtype_code(qkv.dtype), ptr(y), ptr(lse), sp))


def attn_bwd(qkv, y, dy, lse, B, T, n_head, d, dqkv, ws, drop=(0.0, 0), seed_ptr=None, stream=None):
    """Algorithmic FLOPs: twice the forward (dQ, dK, dV, dP; the recomputed S is not counted)."""
    fl = 2.0 * attn_flops(B, T, n_head, d)
    if drop[0] > 0:
        _maybe_timed(stream, "attn_bwd", fl, lambda sp: call(
            "aw_attn_bwd_dropout", ptr(qkv), ptr(y), ptr(dy), ptr(lse), B, T, n_head, d, dtype_code(qkv.dtype),
            ptr(dqkv), ptr(ws), float(drop[0]), int(drop[1]) & 0xFFFFFFFFFFFFFFFF, ptr(seed_ptr), sp))
        return
    _maybe_timed(stream, "attn_bwd", fl, lambda sp: call(
        "aw_attn_bwd", ptr(qkv), ptr(y), ptr(dy), ptr(lse), B, T, n_head, d, dtype_code(qkv.dtype), ptr(dqkv),
        ptr(ws), sp))


# ------------------------------------------------------------------------------ ResBlock BatchNorm
def bn_group_stats(h, G, sums, stream=None):
    N, H = h.shape
    call("aw_bn_group_stats", ptr(h), N, H, int(G), ptr(sums), stream_ptr(stream))


def bn_group_finalize(sums, n, H, G, bn, training, stats, stream=None):
    """stats [4][G][H] from the sums (training) or the running statistics (eval) of nn.BatchNorm1d ``bn``."""
    mom = bn.momentum if bn.momentum is not None else 0.1
    call("aw_bn_group_finalize", ptr(sums) if training else None, int(n), int(H), int(G), ptr(bn.weight),
         ptr(bn.bias), ptr(bn.running_mean), ptr(bn.running_var), ptr(bn.num_batches_tracked) if training else None,
         float(bn.eps), float(mom), int(bool(training)), ptr(stats), stream_ptr(stream))


def bn_apply(h, G, stats, mode, out, op=None, resid=None, drop=(0.0, 0), seed_ptr=None, stream=None):
    N, H = h.shape
    call("aw_bn_apply", ptr(h), N, H, int(G), ptr(stats), int(mode), ptr(resid), float(drop[0]), int(drop[1]),
         ptr(seed_ptr), ptr(out), ptr(op), dtype_code(op.dtype) if op is not None else AW_F32, stream_ptr(stream))


def bn_bwd_reduce(h, G, stats, g_in, sums, drop=(0.0, 0), seed_ptr=None, stream=None):
    N, H = h.shape
    call("aw_bn_bwd_reduce", ptr(h), N, H, int(G), ptr(stats), ptr(g_in), float(drop[0]), int(drop[1]),
         ptr(seed_ptr), ptr(sums), stream_ptr(stream))


def bn_bwd_apply(h, G, stats, g_in, sums, n, training, dh, dgamma=None, dbeta=None, drop=(0.0, 0), seed_ptr=None,
                 stream=None):
    N, H = h.shape
    call("aw_bn_bwd_apply", ptr(h), N, H, int(G), ptr(stats), ptr(g_in), float(drop[0]), int(drop[1]),
         ptr(seed_ptr), ptr(sums), int(n), int(bool(training)), ptr(dh), dtype_code(dh.dtype), ptr(dgamma),
         ptr(dbeta), stream_ptr(stream))


def attn_decode(qkv_new, B, n_new, pos0, n_head, d, kv_cache, y, stream=None):
    """KV-cache attention for n_new rows per sequence at positions pos0..; kv_cache (B, Tmax, 2d)."""
    if kv_cache.dtype != qkv_new.dtype or y.dtype != qkv_new.dtype or kv_cache.shape[-1] != 2 * d:
        raise nat.NativeError("attn_decode: qkv, cache and y share a dtype; cache rows are [K | V] (2d)")
    call("aw_attn_decode", ptr(qkv_new), B, n_new, pos0, n_head, d, dtype_code(qkv_new.dtype), ptr(kv_cache),
         kv_cache.shape[1], ptr(y), stream_ptr(stream))


def ce_fwd(logits, V, y, ignore_index, loss_sum, count, lse, stream=None):
    R = y.numel()
    call("aw_ce_fwd", ptr(logits), R, V, logits.stride(0), ptr(y), int(ignore_index), ptr(loss_sum), ptr(count),
         ptr(lse), stream_ptr(stream))


def ce_bwd(logits, V, y, ignore_index, lse, count, g, dlogits, stream=None):
    R = y.numel()
    call("aw_ce_bwd", ptr(logits), R, V, logits.stride(0), ptr(y), int(ignore_index), ptr(lse), ptr(count), ptr(g),
         ptr(dlogits), dlogits.stride(0), dtype_code(dlogits.dtype), stream_ptr(stream))


def ce_finalize(loss_sum, count, out, stream=None):
    call("aw_ce_finalize", ptr(loss_sum), ptr(count), ptr(out), stream_ptr(stream))
