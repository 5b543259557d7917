"""The fused ResBlock chains (csrc/reschain.hip, aw_res_chain_fwd / aw_res_chain_bwd) against the per-conv GEMM
launches they replace (model/vq_vae_patch_embedd.py:60-74 ResBlock inside CNNBlock :103-110): the encoder's stack
(taps 1: CNNBlock(seperate=True), centre taps) and the decoder's (taps 3: k = 3 convs along 16-token windows, the
implicit conv GEMM with conv_seg 16).

Both paths run the same MFMA sequence per accumulator and the same epilogue operations per element, so every output
is compared BIT FOR BIT: the forward's h / a1 / x / a of every block, the dropout keep bits it writes, and the
backward's gh / masked gx, with dropout on (counter-based masks from a device step counter), at the bench's N = 16384
tokens and at ragged row counts (a partial last 64-row block; a single row / window), for R = 8 / 3 / 1 / 2.  The
unfused launches are themselves checked against torch fp32 and the oracle elsewhere (tests/test_gpu_kernels.py,
tests/test_vqvae_full_batch.py); the last test here runs the whole bf16 VQ-VAE training step both ways at B = 1024
and requires an identical loss and x_hat, and gradients equal up to the order of the atomics that some
weight-gradient launches add their bias sums with.
"""
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


def _conv(taps, d):
    """aw_gemm's implicit conv form of a decoder conv (forward d = 1, input gradient d = -1); {} for the encoder."""
    return dict(conv=(H, SEG, d, 0)) if taps == 3 else {}


def _dgrad_copy(w, taps):
    """The per-conv path's input-gradient operand [(j, o)][i] of a [O][taps*I] forward copy (vqvae.py's dgw)."""
    return w.view(H, taps, H).permute(1, 0, 2).reshape(taps * H, H).contiguous()


def _unfused_fwd(a0, x0, w1, w2, b1, b2, p, seeds, ctr, taps):
    """arcweld/vqvae.py's per-conv launches (the ARCWELD_ENC_CHAIN=0 / ARCWELD_DEC_CHAIN=0 path)."""
    K = _k()
    N = a0.shape[0]
    R = len(w1)
    e = lambda: torch.empty(N, H, device="cuda", dtype=BF)  # noqa: E731
    cv = _conv(taps, 1)
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


@pytest.mark.parametrize("taps", [1, 3])
@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_res_chain_fwd_matches_per_conv_launches_bitwise(taps, case, p):
    K = _k()
    N, R = CASES[taps][case]
    x0 = _rand((N, H), 11)
    a0 = _rand((N, H), 12)
    w1, w2, b1, b2 = _weights(R, 100, taps)
    seeds = [0x1234 + 77 * r for r in range(R)]
    ctr = torch.tensor([5], device="cuda", dtype=torch.int64)
    ref = _unfused_fwd(a0, x0, w1, w2, b1, b2, p, seeds, ctr, taps)
    e = lambda: torch.full((N, H), float("nan"), device="cuda", dtype=BF)  # noqa: E731
    h, a1, x, a = [e() for _ in range(R)], [e() for _ in range(R)], [e() if r < R - 1 else None for r in range(R)], \
        [e() for _ in range(R)]
    pk = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(2 * R)]
    K.res_pack_weights(w1 + w2, pk, taps=taps)
    w1, w2 = pk[:R], pk[R:]
    masks = K.res_dropout_masks_empty(N, R, "cuda") if p > 0 else None
    K.res_chain_fwd(a0, x0, w1, w2, b1, b2, h, a1, x, a, drop=(p, seeds), seed_ptr=ctr, masks=masks, taps=taps)
    torch.cuda.synchronize()
    for nm, got, want in (("h", h, ref[0]), ("a1", a1, ref[1]), ("x", x[:R - 1], ref[2][:R - 1]), ("a", a, ref[3])):
        for r, (g_, w_) in enumerate(zip(got, want)):
            _same(g_, w_, f"{nm}[{r}]")
    if p > 0:   # the keep bits the forward wrote are the standalone mask kernel's
        assert torch.equal(masks, K.res_dropout_masks(N, (p, seeds), ctr))
    # eval form: nothing saved, only the chain's operand outputs
    a_e = [e() for _ in range(R)]
    K.res_chain_fwd(a0, x0, w1, w2, b1, b2, [None] * R, [None] * R, [None] * R, a_e, drop=(p, seeds), seed_ptr=ctr,
                    taps=taps)
    torch.cuda.synchronize()
    for r in range(R):
        _same(a_e[r], ref[3][r], f"eval a[{r}]")


@pytest.mark.parametrize("taps", [1, 3])
@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_res_chain_bwd_matches_per_conv_launches_bitwise(taps, case, p):
    K = _k()
    N, R = CASES[taps][case]
    gx = _rand((N, H), 21, 0.01)
    gxo = _rand((N, H), 22, 0.01)
    hs = [_rand((N, H), 30 + r) for r in range(R)]
    xs = [_rand((N, H), 50 + r) for r in range(R)]
    w1, w2, _, _ = _weights(R, 200, taps)
    seeds = [0x4321 + 13 * r for r in range(R)]
    ctr = torch.tensor([9], device="cuda", dtype=torch.int64)
    e = lambda: torch.empty(N, H, device="cuda", dtype=BF)  # noqa: E731
    cv = _conv(taps, -1)
    # unfused (arcweld/vqvae.py backward, ARCWELD_*_CHAIN=0)
    g_x, g_o = gx, gxo
    ref_gh, ref_go = [None] * R, [None] * R
    for r in reversed(range(R)):
        gh = e()
        K.gemm(g_o, _dgrad_copy(w2[r], taps), N, H, taps * H, b_trans=True, pre=hs[r], C=gh, **cv)
        gxn, gxon = e(), e()
        K.gemm(gh, _dgrad_copy(w1[r], taps), N, H, taps * H, b_trans=True, pre=xs[r], resid=g_x, C=gxn, C2=gxon,
               c2_mode=3 if r > 0 else 2, drop2=(p, seeds[r - 1] if r > 0 else 0), seed_ptr=ctr, **cv)
        ref_gh[r], ref_go[r] = gh, gxon
        g_x, g_o = gxn, gxon
    # chain, on the packed backward weight copies
    wt1 = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(R)]
    wt2 = [torch.empty(H, taps * H, device="cuda", dtype=BF) for _ in range(R)]
    K.res_pack_weights(w1 + w2, None, wt1 + wt2, taps=taps)
    gh_c = [torch.full((N, H), float("nan"), device="cuda", dtype=BF) for _ in range(R)]
    go_c = [torch.full((N, H), float("nan"), device="cuda", dtype=BF) for _ in range(R)]
    masks = K.res_dropout_masks(N, (p, seeds), ctr)
    K.res_chain_bwd(gx, gxo, wt1, wt2, hs, xs, gh_c, go_c, drop_p=p, masks=masks, taps=taps)
    torch.cuda.synchronize()
    for nm, got, want in (("gh", gh_c, ref_gh), ("go", go_c, ref_go)):
        for r in range(R):
            _same(got[r], want[r], f"{nm}[{r}]")


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
    chains and with the per-conv launches: identical losses, x_hat and gradients."""
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
    assert out["0"][0] == out["1"][0]
    assert torch.equal(out["0"][1], out["1"][1])
    # the saved tensors are identical (above), so the gradients differ only by the order of the f32 atomics some
    # weight-gradient launches sum their bias row sums with (run-to-run noise, ~1e-7 relative)
    for n, g0 in out["0"][2].items():
        g1 = out["1"][2][n]
        if n == "reverse_patch_embed.proj.0.bias":   # feeds a train-mode BatchNorm: analytically zero, noise only
            assert g0.abs().max().item() < 1e-5 and g1.abs().max().item() < 1e-5
            continue
        assert (g0 - g1).abs().max().item() <= 1e-5 * g0.abs().max().item() + 1e-12, n
