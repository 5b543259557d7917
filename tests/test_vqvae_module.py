"""VQVAEPatch drop-in: module surface on CPU; fused HIP forward/backward against the reference's golden
fixtures on the GPU (fp32 operands, the default: exact-f32 MFMA; bf16 operands are an explicit opt-in,
arcweld.precision)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import gen
from oracle import vqvae as ov

CASES = {
    "vqvae_small.npz": (dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25), 8,
                        301, 302),
    "vqvae_small_p10.npz": (dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=10), 4,
                            305, 306),
    "vqvae_small_p50.npz": (dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=50), 4,
                            307, 308),
}


def make_model(kw, wseed, device="cpu", batch_norm=False, dropout=0.0):
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=dropout, batch_norm=batch_norm, **kw)
    cfg = ov.VQVAEConfig(batch_norm=batch_norm, **kw)
    sd = ov.det_state_dict(cfg, wseed)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.to(device)


@pytest.mark.parametrize("kw", [dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25),
                                dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=10,
                                     batch_norm=True)])
def test_state_dict_layout_matches_reference(kw):
    from model.vq_vae_patch_embedd import VQVAEPatch
    bn = kw.pop("batch_norm", False)
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, batch_norm=bn, **kw)
    ref = ov.reference_state_dict_shapes(ov.VQVAEConfig(batch_norm=bn, **kw))
    got = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert got == {k: tuple(s) for k, s in ref.items()}
    assert m.enc_out_len == 200 // kw["patch_size"] * 2
    assert m.hparams["hidden_dim"] == kw["hidden_dim"] and m.hparams["patch_size"] == kw["patch_size"]


def test_unsupported_patch_size_raises():
    from model.vq_vae_patch_embedd import VQVAEPatch
    with pytest.raises(NotImplementedError):
        VQVAEPatch(hidden_dim=8, input_dim=2, num_embeddings=4, embedding_dim=4, n_resblocks=1, learning_rate=1e-3,
                   patch_size=20)


@pytest.fixture
def fp32_parity():
    from arcweld.precision import operands
    with operands(torch.float32):
        yield


def _check_grads(m, g, rtol=1e-3):
    for name, p in m.named_parameters():
        ref = g["grad/" + name]
        got = p.grad.detach().cpu().numpy()
        scale = np.abs(ref).max() + 1e-12
        np.testing.assert_allclose(got, ref, rtol=rtol, atol=2e-4 * scale + 1e-7, err_msg=name)


@pytest.mark.gpu
@pytest.mark.parametrize("fname", list(CASES))
def test_vqvae_train_step_parity_fp32(fname, fp32_parity):
    from arcweld.functional import mse_loss
    kw, B, wseed, xseed = CASES[fname]
    g = golden(fname)
    m = make_model(kw, wseed, "cuda")
    m.train()
    x = torch.tensor(gen.windows(xseed, B), device="cuda")
    emb, x_hat, perp = m(x)
    recon = mse_loss(x_hat, x)
    loss = recon + emb
    loss.backward()
    idx = m._last_indices.cpu().numpy()
    assert np.array_equal(idx, g["idx"]), f"{(idx != g['idx']).sum()} index mismatches"
    np.testing.assert_allclose(x_hat.detach().cpu().numpy(), g["x_hat"], rtol=1e-4, atol=1e-4)
    for k, v in (("emb_loss", emb), ("perplexity", perp), ("recon", recon), ("loss", loss)):
        np.testing.assert_allclose(v.item(), g[k], rtol=1e-4, err_msg=k)
    _check_grads(m, g)
    sd = m.state_dict()
    for k in g.files:
        if k.startswith("state/") and "running" in k:
            np.testing.assert_allclose(sd[k[6:]].cpu().numpy(), g[k], rtol=1e-4, atol=1e-5, err_msg=k)
    assert int(sd["reverse_patch_embed.proj.1.num_batches_tracked"]) == 1
    m.eval()
    with torch.no_grad():
        e2, xh2, _ = m(x)
    np.testing.assert_allclose(xh2.cpu().numpy(), g["eval_x_hat"], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_vqvae_batchnorm_resblocks_parity_fp32(fp32_parity):
    """`--batchnorm 1` ResBlocks (vq_vae_patch_embedd.py:60-74): per-token BatchNorm statistics in the encoder
    (its blocks run on every token slice separately), per-channel in the decoder; one train step against the
    reference's golden output, gradients (BN weights and biases included), running statistics and
    num_batches_tracked (S per encoder BN, 1 per decoder BN), then the eval forward on the updated running stats."""
    from arcweld.functional import mse_loss
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
    g = golden("vqvae_small_bn.npz")
    m = make_model(kw, 303, "cuda", batch_norm=True).train()
    x = torch.tensor(gen.windows(304, 8), device="cuda")
    emb, x_hat, perp = m(x)
    recon = mse_loss(x_hat, x)
    loss = recon + emb
    loss.backward()
    assert np.array_equal(m._last_indices.cpu().numpy(), g["idx"])
    np.testing.assert_allclose(x_hat.detach().cpu().numpy(), g["x_hat"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-4)
    _check_grads(m, g)
    sd = m.state_dict()
    for k in g.files:
        if k.startswith("state/"):
            ref = g[k]
            got = sd[k[6:]].cpu().numpy()
            if "num_batches_tracked" in k:
                assert int(got) == int(ref), k
            else:
                np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5, err_msg=k)
    if "eval_x_hat" in g.files:
        m.eval()
        with torch.no_grad():
            _, xh2, _ = m(x)
        np.testing.assert_allclose(xh2.cpu().numpy(), g["eval_x_hat"], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_vqvae_full_size_parity_fp32(fp32_parity):
    from arcweld.functional import mse_loss
    g = golden("vqvae_full_b4.npz")
    kw = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)
    m = make_model(kw, 309, "cuda")
    x = torch.tensor(gen.windows(310, 4), device="cuda")
    emb, x_hat, perp = m(x)
    loss = mse_loss(x_hat, x) + emb
    loss.backward()
    assert np.array_equal(m._last_indices.cpu().numpy(), g["idx"])
    np.testing.assert_allclose(x_hat.detach().cpu().numpy(), g["x_hat"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-4)
    for name, p in m.named_parameters():
        got = p.grad.detach().cpu().numpy()
        if name == "reverse_patch_embed.proj.0.bias":
            # feeds a train-mode BatchNorm: analytically zero, rounding noise on both sides
            assert np.abs(got).max() < 1e-6 and g["gnorm/" + name] < 1e-6, name
            continue
        gn = np.linalg.norm(got.astype(np.float64))
        np.testing.assert_allclose(gn, g["gnorm/" + name], rtol=2e-4, atol=1e-9, err_msg=name)
        # the first 64 elements of the flattened gradient, element by element
        ref = g["gslice/" + name]
        np.testing.assert_allclose(got.reshape(-1)[:64], ref, rtol=1e-3, atol=2e-4 * np.abs(got).max() + 1e-9,
                                   err_msg=name)


@pytest.mark.gpu
def test_vqvae_bf16_mode_tracks_fp32():
    """bf16 MFMA operands (fp32 accumulate) with bf16 residual streams -- what the reference holds under bf16 autocast
    (arcweld/vqvae.py resid_dtype): the codebook indices agree with the fp32 golden on >= 95 % of the tokens (a
    bf16-rounded z may pick the other code of a near tie: here 2 of 128 tokens, both in one window), and every window
    whose tokens all agree reconstructs within bf16 tolerance (5 % of max |x_hat|; measured 0.005 of 0.74)."""
    from arcweld.precision import operands
    with operands(torch.bfloat16):
        kw, B, wseed, xseed = CASES["vqvae_small.npz"]
        g = golden("vqvae_small.npz")
        m = make_model(kw, wseed, "cuda")
        x = torch.tensor(gen.windows(xseed, B), device="cuda")
        emb, x_hat, perp = m(x)
        idx = m._last_indices.cpu().numpy()
    same = idx == g["idx"].reshape(-1)
    assert same.mean() >= 0.95, same.mean()
    whole = same.reshape(B, -1).all(1)
    assert whole.sum() >= B - 2, whole
    err = np.abs(x_hat.detach().cpu().numpy() - g["x_hat"])[whole].max()
    assert err < 5e-2 * np.abs(g["x_hat"]).max(), err


@pytest.mark.gpu
def test_vqvae_dropout_train_step_runs_and_is_seeded():
    kw, B, wseed, xseed = CASES["vqvae_small.npz"]
    m = make_model(kw, wseed, "cuda", dropout=0.1)
    x = torch.tensor(gen.windows(xseed, B), device="cuda")
    torch.manual_seed(3)
    _, a, _ = m(x)
    m._rng_counter.zero_()          # the per-call part of the seed lives on the device
    _, b, _ = m(x)
    assert torch.equal(a, b)
    _, c, _ = m(x)
    assert not torch.equal(a, c)


@pytest.mark.gpu
def test_graphed_steps_match_eager_steps(fp32_parity):
    """Trainer.graphed_step (two captured HIP graphs per step) follows the same trajectory as eager steps:
    same dropout masks (device counter), same RAdam step numbers (device step), same clip."""
    from arcweld.trainer import Trainer
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
    xs = [torch.tensor(gen.windows(700 + i, 16), device="cuda") for i in range(6)]
    runs = []
    for graphed in (False, True):
        m = make_model(kw, 301, "cuda", dropout=0.1).train()
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        losses = []
        for x in xs:
            if graphed:
                losses.append(float(tr.graphed_step(m, x, 1.0)))
            else:
                losses.append(float(tr.micro_step(m, x, 0, 1.0)))
                tr.optimizer_step(m)
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}, tr.global_step))
    (l0, s0, n0), (l1, s1, n1) = runs
    assert n0 == n1 == 6
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    for k in s0:
        torch.testing.assert_close(s1[k].float(), s0[k].float(), rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("fname", ["vqvae_small.npz", "vqvae_small_p10.npz"])
def test_fused_train_step_matches_golden_and_split_point_is_final(fname, fp32_parity):
    """fused_train_step (no autograd; what the captured step runs) gives the golden loss and gradients, and at its
    mid_hook every gradient from backward_split_parameter() on is already final while the ones before it are
    untouched -- the invariant the overlapped decoder-side all-reduce relies on."""
    kw, B, wseed, xseed = CASES[fname]
    g = golden(fname)
    m = make_model(kw, wseed, "cuda").train()
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    x = torch.tensor(gen.windows(xseed, B), device="cuda")
    names = [n for n, _ in m.named_parameters()]
    params = list(m.parameters())
    cut = next(i for i, p in enumerate(params) if p is m.backward_split_parameter())
    snap = []
    loss = m.fused_train_step(x, 1.0, mid_hook=lambda: snap.append([p.grad.clone() for p in params]))
    assert len(snap) == 1
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-4)
    assert np.array_equal(m._last_indices.cpu().numpy(), g["idx"])
    _check_grads(m, g)
    for i, (n, p) in enumerate(zip(names, params)):
        if i >= cut:
            assert torch.equal(snap[0][i], p.grad), n
        else:
            assert not snap[0][i].any(), n


@pytest.mark.gpu
def test_full_size_bf16_grads_agree_across_gemm_tiles():
    """Full-size model, bf16 operands: the automatic tile policy (256x128 three-stage pipeline for the grouped
    weight gradients) and every launch forced onto 128x128 tiles give the same step up to summation order."""
    from arcweld import _native
    from arcweld.precision import set_operand_dtype
    kw = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)
    m = make_model(kw, 311, "cuda").train()
    x = torch.tensor(gen.windows(312, 64), device="cuda")
    grads = {}
    try:
        set_operand_dtype(torch.bfloat16)
        for bm in (0, 128):
            _native.call("aw_gemm_set_tile", bm)
            m.zero_grad()
            emb, x_hat, _ = m(x)
            (torch.nn.functional.mse_loss(x_hat, x) + emb).backward()
            grads[bm] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    finally:
        _native.call("aw_gemm_set_tile", 0)
        set_operand_dtype(None)
    for n in grads[0]:
        if n == "reverse_patch_embed.proj.0.bias":
            continue   # feeds a train-mode BatchNorm: its gradient is zero up to rounding noise
        a, b = grads[0][n], grads[128][n]
        rel = ((a - b).norm() / (b.norm() + 1e-20)).item()
        assert rel < 2e-3, (n, rel)


@pytest.mark.gpu
def test_trainer_centre_tap_layout_matches_dense_layout(fp32_parity, monkeypatch):
    """The Trainer stores the encoder conv weights tap-major (side taps out of the optimizer); three steps give the
    same parameters as the dense layout, and the side taps stay at their initial values."""
    from arcweld.optim import RAdam
    from arcweld.trainer import Trainer
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
    xs = [torch.tensor(gen.windows(720 + i, 16), device="cuda") for i in range(3)]
    out = []
    for declare in (True, False):
        if not declare:
            monkeypatch.setattr(RAdam, "declare_centre_tap", lambda self, ps: None)
        m = make_model(kw, 301, "cuda").train()
        init = {k: v.detach().clone() for k, v in m.state_dict().items()}
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        assert (not m.encoder[0].shared_conv[0].block[1].weight.is_contiguous()) == declare
        for x in xs:
            tr.micro_step(m, x, 0, 1.0)
            tr.optimizer_step(m)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        for k, v in sd.items():
            if k.startswith("encoder.0.") and k.endswith("weight"):
                assert torch.equal(v[:, :, 0], init[k][:, :, 0]) and torch.equal(v[:, :, 2], init[k][:, :, 2]), k
        out.append(sd)
    for k in out[0]:
        torch.testing.assert_close(out[0][k].float(), out[1][k].float(), rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("batch_norm", [False, True])
def test_trainer_tap_major_decoder_layout_matches_dense_layout(fp32_parity, monkeypatch, batch_norm):
    """The Trainer stores the decoder k = 3 conv weights tap-major ((O, 3, I) segments: contiguous weight-gradient
    atomics, plain-cast forward operands); three steps with dropout give the same parameters as the reference's dense
    (O, I, 3) layout, and the state_dict keeps the reference's shapes."""
    from arcweld.optim import RAdam
    from arcweld.trainer import Trainer
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
    xs = [torch.tensor(gen.windows(730 + i, 16), device="cuda") for i in range(3)]
    out = []
    for declare in (True, False):
        if not declare:
            monkeypatch.setattr(RAdam, "declare_tap_major", lambda self, ps: None)
        m = make_model(kw, 302, "cuda", batch_norm=batch_norm, dropout=0.1).train()
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        w = m.decoder[1].shared_conv[0].block[1].weight
        assert (not w.is_contiguous()) == declare and w.shape == (64, 64, 3)
        for x in xs:
            tr.micro_step(m, x, 0, 1.0)
            tr.optimizer_step(m)
        out.append({k: v.detach().clone() for k, v in m.state_dict().items()})
    for k in out[0]:
        torch.testing.assert_close(out[0][k].float(), out[1][k].float(), rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.gpu
def test_batchnorm_model_tokenizes_and_trains_graphed(fp32_parity):
    """BatchNorm ResBlocks on the other entry points: the fused tokenization gives the train-step indices of the
    golden (batch statistics in train mode), the standalone encoder modules agree with it, and captured steps
    follow eager steps."""
    from arcweld.trainer import Trainer
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
    g = golden("vqvae_small_bn.npz")
    m = make_model(kw, 303, "cuda", batch_norm=True).train()
    x = torch.tensor(gen.windows(304, 8), device="cuda")
    ids = m.encode_ids(x)
    assert np.array_equal(ids.reshape(-1).cpu().numpy(), g["idx"])
    m2 = make_model(kw, 303, "cuda", batch_norm=True).eval()
    with torch.no_grad():
        z = m2.encoder(m2.patch_embed(x))           # standalone modules (latentspace_dataloader.py:154-161)
        _, _, _, _, idx2 = m2.vector_quantization(z)
    ids2 = m2.encode_ids(x)
    assert torch.equal(idx2.reshape(-1).cpu(), ids2.reshape(-1).cpu())
    xs = [torch.tensor(gen.windows(760 + i, 16), device="cuda") for i in range(4)]
    runs = []
    for graphed in (False, True):
        mm = make_model(kw, 303, "cuda", batch_norm=True, dropout=0.1).train()
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(mm)
        for xx in xs:
            if graphed:
                tr.graphed_step(mm, xx, 1.0)
            else:
                tr.micro_step(mm, xx, 0, 1.0)
                tr.optimizer_step(mm)
        runs.append({k: v.detach().clone() for k, v in mm.state_dict().items()})
    for k in runs[0]:
        torch.testing.assert_close(runs[1][k].float(), runs[0][k].float(), rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.gpu
def test_batchnorm_single_window_training_batch_raises(fp32_parity):
    """--batchnorm 1 with a ragged last batch of ONE window: the encoder BN groups hold one value per channel;
    torch BatchNorm1d raises ValueError in training (eval mode, on running statistics, is fine)."""
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=25)
    m = make_model(kw, 303, "cuda", batch_norm=True).train()
    x = torch.tensor(gen.windows(304, 1), device="cuda")
    with pytest.raises(ValueError, match="more than 1 value per channel"):
        m(x)
    m.eval()
    with torch.no_grad():
        _, xh, _ = m(x)
    assert torch.isfinite(xh).all()


@pytest.mark.gpu
def test_graphed_fit_logs_the_loss_history(fp32_parity):
    """Trainer(hip_graphs=True).fit records (step, loss) every log_every_n_steps from the captured step's static
    loss tensor, as the eager path does."""
    from arcweld.data import DeviceBatches
    from arcweld.trainer import Trainer
    kw = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=1, patch_size=25)
    data = torch.tensor(gen.windows(731, 64), device="cuda")
    hist = []
    for graphs in (False, True):
        m = make_model(kw, 301, "cuda").train()
        tr = Trainer(gradient_clip_val=0.7, hip_graphs=graphs, log_every_n_steps=2, max_epochs=1)
        tr.fit(m, train_dataloaders=DeviceBatches(data, 8, shuffle=False))
        assert tr.global_step == 8
        hist.append(tr.history)
    assert [h[0] for h in hist[1]] == [h[0] for h in hist[0]] == [2, 4, 6, 8]
    np.testing.assert_allclose([h[1] for h in hist[1]], [h[1] for h in hist[0]], rtol=1e-4)
