"""The fused ResBlock chains (csrc/reschain.hip, aw_res_chain_fwd / aw_res_chain_bwd) against the per-conv GEMM
launches they replace (model/vq_vae_patch_embedd.py:60-74 ResBlock inside CNNBlock :103-110): the encoder's stack
(taps 1: CNNBlock(seperate=True), centre taps) and the decoder's (taps 3: k = 3 convs along 16-token windows, the
implicit conv GEMM with conv_seg 16).

Round 6: in place of the unfused path's saved h and x the forward saves GELU'(h) and GELU'(x') (the backward then
evaluates no transcendental).  Both paths run the same MFMA sequence per accumulator and the same epilogue operations
per element, so the forward's operand outputs a1 / a of every block and the dropout keep bits it writes are compared
BIT FOR BIT with the per-conv launches.  The saved derivatives, and the backward that multiplies by them, are checked
against a torch fp32 restatement of the same bf16 recursion -- the same inputs and weights, bf16 roundings at the
same points, the dropout keep bits from the kernels' counter hash restated in numpy -- where only the f32
accumulation order differs (block by block, each block restarting from the chain's own operand).  Every case runs with
dropout on and off (counter-based masks from a device step counter), at the bench's N = 16384 tokens and at ragged
row counts (a partial last 64-row block; a single row / window), for R = 8 / 3 / 1 / 2.  The unfused launches are
themselves checked against torch fp32 and the oracle elsewhere (tests/test_gpu_kernels.py,
tests/test_vqvae_full_batch.py); the last test here runs the whole bf16 VQ-VAE training step both ways at B = 1024:
identical loss and x_hat, gradients within the bf16 rounding of the saved derivatives.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

H = 512
SEG = 16
BF = torch.bfloat16
CASES = {1: [(16384, 8), (1000, 3), (64, 1), (1, 2)], 3: [(16384, 8), (1008, 3), (64, 1), (16, 2)]}


def _k():
    from arcweld import kernels as K
    return K


def _rand(shape, seed, scale=1.0, dtype=BF):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).cuda()


def _weights(R, seed, taps):
    """R (conv1, conv2) forward operand copies [O][taps*I] (column j*I + i) and biases."""
    sc = (taps * H) ** -0.5
    w1 = [_rand((H, taps * H), seed + 10 * r, sc) for r in range(R)]
    w2 = [_rand((H, taps * H), seed + 10 * r + 1, sc) for r in range(R)]
    b1 = [_rand((H,), seed + 10 * r + 2, 0.1, torch.float32) for r in range(R)]
    b2 = [_rand((H,), seed + 10 * r + 3, 0.1, torch.float32) for r in range(R)]
    return w1, w2, b1, b2


def _gemm_conv(taps, d):
    """aw_gemm's implicit conv form of a decoder conv (forward d = 1, input gradient d = -1); {} for the encoder."""
    return dict(conv=(H, SEG, d, 0)) if taps == 3 else {}


def _unfused_fwd(a0, x0, w1, w2, b1, b2, p, seeds, ctr, taps):
    """arcweld/vqvae.py's per-conv launches (the ARCWELD_ENC_CHAIN=0 / ARCWELD_DEC_CHAIN=0 path)."""
    K = _k()
    N = a0.shape[0]
    R = len(w1)
    e = lambda: torch.empty(N, H, device="cuda", dtype=BF)  # noqa: E731
    cv = _gemm_conv(taps, 1)
    xs, a0s, hs, a1s = [x0], [a0], [], []
    for r in range(R):
        h, a1 = e(), e()
        K.gemm(a0s[r], w1[r], N, H, taps * H, bias=b1[r], C=h, C2=a1, c2_mode=1, **cv)
        if r < R - 1:
            xn, an = e(), e()
            K.gemm(a1, w2[r], N, H, taps * H, bias=b2[r], drop=(p, seeds[r]), seed_ptr=ctr, resid=xs[r], C=xn, C2=an,
                   c2_mode=1, **cv)
        else:
            xn, an = None, e()
            K.gemm(a1, w2[r], N, H, taps * H, bias=b2[r], drop=(p, seeds[r]), seed_ptr=ctr, resid=xs[r], C=an, **cv)
        xs.append(xn)
        a0s.append(an)
        hs.append(h)
        a1s.append(a1)
    return hs, a1s, xs[1:], a0s[1:]


def _same(got, want, what):
    gi, wi = got.view(torch.int16), want.view(torch.int16)
    assert torch.equal(gi, wi), f"{what}: {int((gi != wi).sum())} elements differ"


def _gelu_grad(v):
    """GELU'(v) of the erf form, torch fp32 (the kernels' Abramowitz-Stegun Phi is within 2.5e-7 of it)."""
    v = v.float()
    return 0.5 * (1.0 + torch.erf(v * 0.7071067811865476)) + v * 0.3989422804014327 * torch.exp(-0.5 * v * v)


def _seed_mix(salt, ctr):
    """aw_seed_mix_value (csrc/common.h), as oracle/residual_vq.py restates it."""
    M = (1 << 64) - 1
    z = (salt ^ ((ctr * 0xD1B54A32D192ED03 + 0x8CB92BA72F3D8DD7) & M)) & M
    z = ((z ^ (z >> 32)) * 0xD6E8FEB86659FD93) & M
    return z ^ (z >> 32)


def _drop_scale(N, seed, ctr, p):
    """The dropout scale of element (row, c) under aw_gemm's epilogue mask (common.h aw_dropout_scale4: splitmix64 of
    seed_mix(seed, ctr) on group (row * H + c) >> 2, 16-bit slice e & 3, dropped iff < round(p * 65536)), numpy."""
    e = np.arange(N * H, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(_seed_mix(seed, ctr)) + (e // np.uint64(4) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> (np.uint64(16) * (e & np.uint64(3)))) & np.uint64(0xFFFF)
    keep = u >= np.uint64(int(p * 65536 + 0.5))
    return torch.tensor(np.where(keep, np.float32(1.0 / (1.0 - p)), np.float32(0.0)).reshape(N, H)).cuda()


def _convT(w, v, taps):
    """The chain backward's input-gradient conv in torch fp32: out[t] = sum_j W_j^T v[t - j + 1] within each 16-row
    window (taps 3), or W^T v[t] (taps 1); w the [O][taps*I] forward copy (column j*I + i)."""
    W = w.float().view(H, taps, H)
    if taps == 1:
        return v @ W[:, 0, :]
    N = v.shape[0]
    vw = v.view(N // SEG, SEG, H)
    out = torch.zeros_like(vw)
    for j in range(3):
        sh = torch.zeros_like(vw)
        d = 1 - j                      # out[t] reads v[t + d]
        if d > 0:
            sh[:, :SEG - d] = vw[:, d:]
        elif d < 0:
            sh[:, -d:] = vw[:, :SEG + d]
        else:
            sh = vw
        out += sh @ W[:, j, :]
    return out.view(N, H)


def _conv(w, v, taps):
    """The chain forward's conv in torch fp32: out[t] = sum_j W_j v[t + j - 1] within each 16-row window (taps 3), or
    W v[t] (taps 1); w the [O][taps*I] forward copy (column j*I + i)."""
    W = w.float().view(H, taps, H)
    if taps == 1:
        return v @ W[:, 0, :].t()
    N = v.shape[0]
    vw = v.view(N // SEG, SEG, H)
    out = torch.zeros_like(vw)
    for j in range(3):
        d = j - 1                      # out[t] reads v[t + d]
        sh = torch.zeros_like(vw)
        if d > 0:
            sh[:, :SEG - d] = vw[:, d:]
        elif d < 0:
            sh[:, -d:] = vw[:, :SEG + d]
        else:
            sh = vw
        out += sh @ W[:, j, :].t()
    return out.view(N, H)


def _gelu(v):
    return v * 0.5 * (1.0 + torch.erf(v * 0.7071067811865476))


def _within_one_step(got, want, what, steps=1):
    """Every element within `steps` bf16 steps of the reference (each at most 2^-7 of the value, the coarsest bf16
    spacing) plus 2^-12 of the tensor's rms for values near zero: the two sides differ in f32 summation order only."""
    g_, w_ = got.float(), want.float()
    rms = float(w_.pow(2).mean().sqrt())
    err = (g_ - w_).abs()
    bad = err > steps * 2.0 ** -7 * w_.abs() + 2.0 ** -12 * rms
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements off, max err {float(err.max()):.3g} (rms {rms:.3g})"
    return float((err > 0).float().mean())


@pytest.mark.parametrize("taps", [1, 3])
@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_res_chain_fwd_matches_torch_fp32_recursion(taps, case, p):
    """a1 / a (x_R for the last block) and the keep bits: the per-conv launches' bit for bit.  The saved derivatives
    against torch fp32 on the same bf16 operands: dh = bf16(GELU'(h)), h = conv(W1, a) + b1; dx = bf16(GELU'(x')),
    x' = x + Dropout(conv(W2, a1) + b2)."""
    K = _k()
    N, R = CASES[taps][case]
    x0 = _rand((N, H), 11)
    a0 = _rand((N, H), 12)
    w1, w2, b1, b2 = _weights(R, 100, taps)
    seeds = [0x1234 + 77 * r for r in range(R)]
    ctr = torch.tensor([5], device="cuda", dtype=torch.int64)
    e = lambda: torch.full((N, H), float("nan"), device="cuda", dtype=BF)  # noqa: E731
    dh, a1, dx, a = [e() for _ in range(R)], [e() for _ in range(R)], [e() if r < R - 1 else None for r in range(R)], \
        [e() for _ in range(R)]
    pk = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(2 * R)]
    K.res_pack_weights(w1 + w2, pk, taps=taps)
    masks = K.res_dropout_masks_empty(N, R, "cuda") if p > 0 else None
    K.res_chain_fwd(a0, x0, pk[:R], pk[R:], b1, b2, dh, a1, dx, a, drop=(p, seeds), seed_ptr=ctr, masks=masks,
                    taps=taps)
    torch.cuda.synchronize()
    if p > 0:   # the keep bits the forward wrote are the standalone mask kernel's
        assert torch.equal(masks, K.res_dropout_masks(N, (p, seeds), ctr))
    # the operands are the per-conv launches' bit for bit (same MFMA sequence, same epilogue operations)
    ref = _unfused_fwd(a0, x0, w1, w2, b1, b2, p, seeds, ctr, taps)
    for r in range(R):
        _same(a1[r], ref[1][r], f"a1[{r}]")
        _same(a[r], ref[3][r], f"a[{r}]")
    # the saved derivatives against torch fp32, block by block: h from the chain's own operand a_r (bit for bit the
    # per-conv one), x' from the per-conv path's residual stream x_r (bit for bit the chain's: the same operations)
    for r in range(R):
        a_in = a0.float() if r == 0 else a[r - 1].float()
        h = _conv(w1[r], a_in, taps) + b1[r]
        _within_one_step(dh[r], _gelu_grad(h).to(BF), f"GELU'(h)[{r}]")
        if r < R - 1:
            t = _conv(w2[r], a1[r].float(), taps) + b2[r]
            if p > 0:
                t = t * _drop_scale(N, seeds[r], 5, p)
            xf = t + (x0.float() if r == 0 else ref[2][r - 1].float())
            _within_one_step(dx[r], _gelu_grad(xf).to(BF), f"GELU'(x)[{r}]")
    # eval form: nothing saved but the operands, the same values
    a1_e, a_e = [e() for _ in range(R)], [e() for _ in range(R)]
    K.res_chain_fwd(a0, x0, pk[:R], pk[R:], b1, b2, [None] * R, a1_e, [None] * R, a_e, drop=(p, seeds), seed_ptr=ctr,
                    taps=taps)
    torch.cuda.synchronize()
    for r in range(R):
        _same(a_e[r], a[r], f"eval a[{r}]")
        _same(a1_e[r], a1[r], f"eval a1[{r}]")


@pytest.mark.parametrize("taps", [1, 3])
@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_res_chain_bwd_matches_torch_fp32_recursion(taps, case, p):
    """gh_r = bf16(convT(W2_r, go_r) * dh_r), v = convT(W1_r, gh_r) * GELU'(x_r) + gx_{r+1} (GELU'(x_r) = the saved dx_r,
    for r = 0 evaluated from x_0), gx_r = bf16(v), go_r = bf16(v * mask_{r-1}) (r > 0) or gx_0: torch fp32 on the same
    bf16 inputs and weights, rounding where the kernel rounds, block by block from the chain's own operand: the two
    sides accumulate in a different order (f32), so an element may land one bf16 step apart."""
    K = _k()
    N, R = CASES[taps][case]
    gx = _rand((N, H), 21, 0.01)
    gxo = _rand((N, H), 22, 0.01)
    x0 = _rand((N, H), 50)
    dh = [_gelu_grad(_rand((N, H), 30 + r)).to(BF) for r in range(R)]
    dx = [None] + [_gelu_grad(_rand((N, H), 50 + r)).to(BF) for r in range(1, R)]
    w1, w2, _, _ = _weights(R, 200, taps)
    seeds = [0x4321 + 13 * r for r in range(R)]
    ctr = torch.tensor([9], device="cuda", dtype=torch.int64)
    # chain, on the packed backward weight copies
    wt1 = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(R)]
    wt2 = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(R)]
    K.res_pack_weights(w1 + w2, None, wt1 + wt2, taps=taps)
    gh_c = [torch.full((N, H), float("nan"), device="cuda", dtype=BF) for _ in range(R)]
    go_c = [torch.full((N, H), float("nan"), device="cuda", dtype=BF) for _ in range(R)]
    masks = K.res_dropout_masks(N, (p, seeds), ctr)
    K.res_chain_bwd(gx, gxo, wt1, wt2, dh, x0, dx, gh_c, go_c, drop_p=p, masks=masks, taps=taps)
    torch.cuda.synchronize()
    # torch fp32 restatement; gmax: elementwise running max of |gx| over the blocks so far (the scale of the rounding
    # drift the reference's own residual gradient can carry)
    gr, go = gx.float(), gxo
    gmax = gr.abs()
    for r in reversed(range(R)):
        gh = (_convT(w2[r], go.float(), taps) * dh[r].float()).to(BF)
        ag = dx[r].float() if r > 0 else _gelu_grad(x0)
        v = _convT(w1[r], gh_c[r].float(), taps) * ag + gr
        gr = v.to(BF).float()
        sc = _drop_scale(N, seeds[r - 1], 9, p) if (r > 0 and p > 0) else None
        go = (v * sc).to(BF) if sc is not None else v.to(BF)
        _within_one_step(gh_c[r], gh, f"gh[{r}]")
        # the residual gradient gx_r never leaves the chain, so the reference carries its own, which may drift from
        # the chain's by up to one step of ITS earlier magnitudes per block it passed (one rounding each, and a later
        # sum may cancel most of the value): go within one step of itself plus that many steps of the running max of
        # |gx| (times the dropout scale)
        gmax = torch.maximum(gmax, gr.abs())
        drift = (R - r) * 2.0 ** -7 * gmax * (sc if sc is not None else 1.0)
        g_, w_ = go_c[r].float(), go.float()
        err = (g_ - w_).abs()
        bad = err > 2.0 ** -7 * w_.abs() + drift + 2.0 ** -12 * float(w_.pow(2).mean().sqrt())
        assert not bool(bad.any()), f"go[{r}]: {int(bad.sum())} elements off, max err {float(err.max()):.3g}"
        # the next block starts from the chain's go (a check per block, not of an accumulated drift); the residual
        # gradient gx_r is no output of the chain for r > 0, so that one stays the reference's
        go = go_c[r]


def _packed_ref(A):
    """The documented packed layout (include/arcweld_amd.h aw_res_pack_weights) of a [512][K] matrix, in torch:
    block (m / 16, k / 32) holds lane l = m % 16 + 16 ((k % 32) / 8), element k % 8."""
    Kd = A.shape[1]
    return A.reshape(32, 16, Kd // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(512, Kd)


@pytest.mark.parametrize("taps", [1, 3])
def test_res_pack_weights_layout(taps):
    K = _k()
    src = [_rand((H, taps * H), 70 + i) for i in range(3)]
    fwd = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(3)]
    bwd = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(3)]
    K.res_pack_weights(src, fwd, bwd, taps=taps)
    only_bwd = [torch.zeros(H, taps * H, device="cuda", dtype=BF) for _ in range(3)]
    K.res_pack_weights(src, None, only_bwd, taps=taps)
    torch.cuda.synchronize()
    for s_, f_, b_, o_ in zip(src, fwd, bwd, only_bwd):
        assert torch.equal(f_, _packed_ref(s_))
        # backward operand A[i][(j, o)] = W[o][j * 512 + i]
        assert torch.equal(b_, _packed_ref(s_.view(H, taps, H).permute(2, 1, 0).reshape(H, taps * H)))
        assert torch.equal(o_, b_)


def test_vqvae_b1024_bf16_step_chain_equals_per_conv(monkeypatch):
    """The whole bf16 VQ-VAE train step (B = 1024, dropout 0.1: every encoder and decoder mask in play) with both
    chains and with the per-conv launches: identical loss and x_hat, gradients to bf16 rounding."""
    from model.vq_vae_patch_embedd import VQVAEPatch

    from arcweld.functional import mse_loss
    from arcweld.precision import operands
    from oracle import gen
    from oracle import vqvae as ov

    kw = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)
    sd = ov.det_state_dict(ov.VQVAEConfig(**kw), 31)
    x = torch.tensor(gen.windows(32, 1024), device="cuda")
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("ARCWELD_ENC_CHAIN", mode)
        monkeypatch.setenv("ARCWELD_DEC_CHAIN", mode)
        m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.1, batch_norm=False, **kw)
        m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
        m = m.cuda().train()
        with operands(torch.bfloat16):
            emb, x_hat, perp = m(x)
            loss = mse_loss(x_hat, x) + emb
            loss.backward()
        torch.cuda.synchronize()
        out[mode] = (loss.item(), x_hat.detach().clone(), {n: p.grad.detach().clone() for n, p in m.named_parameters()})
    # the forward is bit for bit the unfused one; the backward multiplies by GELU' of the f32 pre-activations rounded to
    # bf16 (the unfused one: GELU' of the bf16 pre-activations), so the gradients agree to bf16 rounding: within 1 % of
    # each tensor's norm (the bf16 mode tracks fp32 at 5 %: tests/test_vqvae_full_batch.py)
    assert out["0"][0] == out["1"][0]
    assert torch.equal(out["0"][1], out["1"][1])
    for n, g0 in out["0"][2].items():
        g1 = out["1"][2][n]
        if n == "reverse_patch_embed.proj.0.bias":   # feeds a train-mode BatchNorm: analytically zero, noise only
            assert g0.abs().max().item() < 1e-5 and g1.abs().max().item() < 1e-5
            continue
        if g0.norm() == 0:
            assert g1.norm() == 0, n
            continue
        rel = float((g0 - g1).norm() / g0.norm())
        assert rel <= 1e-2, f"{n}: {rel:.3g}"
