"""MyTransformerDecoder drop-in: module surface / optimizer groups on CPU; the fused HIP forward/backward against
the reference's golden fixtures on the GPU (fp32 parity mode -> exact-f32 MFMA; logits within 1e-4)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import decoder as od
from oracle import gen

SMALL = dict(d_model=64, n_classes=34, seq_len=33, n_blocks=2)
FULL = dict(d_model=512, n_classes=514, seq_len=321, n_blocks=8)
CASES = [("decoder_small.npz", SMALL, 4, 4, 401, 402, False),
         ("decoder_small_bias.npz", SMALL, 4, 3, 403, 404, True)]


def make_model(kw, n_head, wseed, bias=False, device="cpu", res_dropout=0.0):
    from model.transformer_decoder import MyTransformerDecoder
    m = MyTransformerDecoder(n_head=n_head, res_dropout=res_dropout, att_dropout=0.0, class_h_bias=bias, **kw)
    sd = od.det_state_dict(wseed, class_h_bias=bias, **kw)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.to(device)


def inputs(B, T, V, xseed, device="cpu"):
    x = gen.randint(xseed, (B, T), 0, V)
    y = gen.randint(xseed + 1, (B, T), 0, V)
    y[:, -3:] = -1
    cond = gen.randint(xseed + 2, (B,), 0, 2)
    return tuple(torch.tensor(a, device=device) for a in (x, y, cond))


@pytest.mark.parametrize("kw,bias", [(SMALL, False), (SMALL, True), (FULL, False)])
def test_state_dict_layout_matches_reference(kw, bias):
    from model.transformer_decoder import MyTransformerDecoder
    m = MyTransformerDecoder(n_head=4, class_h_bias=bias, **kw)
    ref = od.decoder_state_dict_shapes(class_h_bias=bias, **kw)
    got = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert got == {k: tuple(s) for k, s in ref.items()}
    assert m.hparams["d_model"] == kw["d_model"] and m.hparams["n_classes"] == kw["n_classes"]


def test_optimizer_groups_match_reference():
    """Linear weights decayed (0.1), biases / LayerNorm / Embedding not; betas (0.9, 0.95)."""
    m = make_model(SMALL, 4, 401)
    opt = m.configure_optimizers()
    names = {id(p): n for n, p in m.named_parameters()}
    decay = sorted(names[id(p)] for p in opt.param_groups[0]["params"])
    no_decay = sorted(names[id(p)] for p in opt.param_groups[1]["params"])
    assert opt.param_groups[0]["weight_decay"] == 0.1 and opt.param_groups[1]["weight_decay"] == 0.0
    assert opt.param_groups[0]["betas"] == (0.9, 0.95)
    assert all(n.endswith("weight") and "ln_" not in n and "embedding" not in n for n in decay)
    assert "lm_head.weight" in decay and "transformer.h.0.mlp.c_fc.weight" in decay
    assert "embedding.latent_embedding.weight" in no_decay and "transformer.ln_f.weight" in no_decay
    assert len(decay) + len(no_decay) == len(names)


def test_active_parameters_follow_task():
    m = make_model(SMALL, 4, 401)
    gen_names = {n for n, p in m.named_parameters() if any(p is q for q in m.active_parameters())}
    assert "lm_head.weight" in gen_names and not any(n.startswith("class_head") for n in gen_names)
    m.switch_to_classification()
    cls_names = {n for n, p in m.named_parameters() if any(p is q for q in m.active_parameters())}
    assert "lm_head.weight" not in cls_names and "class_head.linear_1.weight" in cls_names


@pytest.fixture
def fp32_parity():
    from arcweld.precision import operands
    with operands(torch.float32):
        yield


def _step(m, task, batch):
    x, y, cond = batch
    m.zero_grad(set_to_none=True)
    if task == "gen":
        m.switch_to_generate()
        loss, logits, _ = m.step_task_gen((x, cond, y))
    else:
        m.switch_to_classification()
        loss, logits, _ = m.step_task_class((x, cond, y))
    loss.backward()
    return loss, logits


@pytest.mark.gpu
@pytest.mark.parametrize("fname,kw,n_head,B,wseed,xseed,bias", CASES)
def test_train_step_parity_fp32(fp32_parity, fname, kw, n_head, B, wseed, xseed, bias):
    g = golden(fname)
    m = make_model(kw, n_head, wseed, bias, "cuda").train()
    batch = inputs(B, kw["seq_len"], kw["n_classes"], xseed, "cuda")
    for t in ("gen", "cls"):
        loss, logits = _step(m, t, batch)
        np.testing.assert_allclose(logits.detach().cpu().numpy(), g[f"{t}/logits"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(loss.item(), g[f"{t}/loss"], rtol=1e-5)
        got = sorted(n for n, p in m.named_parameters() if p.grad is not None)
        assert got == sorted(g[f"{t}/grad_names"].tolist())
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            ref = g[f"{t}/grad/{n}"]
            np.testing.assert_allclose(p.grad.cpu().numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max() + 1e-7,
                                       err_msg=f"{t} {n}")


@pytest.mark.gpu
def test_train_step_parity_full_size_fp32(fp32_parity):
    g = golden("decoder_full_b2.npz")
    m = make_model(FULL, 8, 405, device="cuda").train()
    batch = inputs(2, 321, 514, 406, "cuda")
    for t in ("gen", "cls"):
        loss, logits = _step(m, t, batch)
        lg = logits.detach().cpu().numpy()
        if t == "gen":
            np.testing.assert_allclose(lg[:, :, :32], g["gen/logits_slice"], rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(lg[:, -1, :], g["gen/logits_lastrow"], rtol=1e-4, atol=1e-4)
        else:
            np.testing.assert_allclose(lg, g["cls/logits"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(loss.item(), g[f"{t}/loss"], rtol=1e-5)
        for n, p in m.named_parameters():
            if p.grad is None:
                continue
            gn = np.linalg.norm(p.grad.double().cpu().numpy())
            np.testing.assert_allclose(gn, g[f"{t}/gnorm/{n}"], rtol=2e-4, err_msg=f"{t} {n}")
            sl = g[f"{t}/gslice/{n}"]
            np.testing.assert_allclose(p.grad.reshape(-1)[:64].cpu().numpy(), sl, rtol=2e-3,
                                       atol=2e-4 * np.abs(sl).max() + 1e-7, err_msg=f"{t} {n}")


@pytest.mark.gpu
def test_eval_forward_matches_train_forward_without_dropout(fp32_parity):
    g = golden("decoder_small.npz")
    m = make_model(SMALL, 4, 401, device="cuda").eval()
    x, y, cond = inputs(4, 33, 34, 402, "cuda")
    with torch.no_grad():
        logits = m(x)
        cls = m(x, generate=False)
    np.testing.assert_allclose(logits.cpu().numpy(), g["gen/logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(cls.cpu().numpy(), g["cls/logits"], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_bf16_tracks_fp32():
    """bf16 MFMA operands (the --precision bf16 opt-in), fp32 accumulation, track the fp32 step."""
    from arcweld.precision import operands
    m = make_model(FULL, 8, 405, device="cuda").train()
    batch = inputs(2, 321, 514, 406, "cuda")
    with operands(torch.float32):
        l32, lg32 = _step(m, "gen", batch)
        g32 = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    with operands(torch.bfloat16):
        l16, lg16 = _step(m, "gen", batch)
    assert abs(l16.item() - l32.item()) < 2e-2 * abs(l32.item())
    err = (lg16 - lg32).abs().max().item()
    assert err < 5e-2 * lg32.abs().max().item() + 1e-2
    for n, p in m.named_parameters():
        if p.grad is None:
            continue
        rel = ((p.grad - g32[n]).norm() / (g32[n].norm() + 1e-12)).item()
        assert rel < 5e-2, (n, rel)


@pytest.mark.gpu
def test_dropout_seeded_and_active(fp32_parity):
    m = make_model(SMALL, 4, 401, device="cuda", res_dropout=0.1).train()
    x, y, cond = inputs(4, 33, 34, 402, "cuda")
    a = m(x).detach()
    b = m(x).detach()
    assert not torch.equal(a, b)                 # fresh mask per call
    m._rng_counter.zero_()
    assert torch.equal(m(x).detach(), a)         # the per-call part of the seed is the device counter
    m.eval()
    c = m(x).detach()
    d = m(x).detach()
    assert torch.equal(c, d)


@pytest.mark.gpu
def test_generate_greedy_matches_oracle_argmax(fp32_parity):
    sd = od.det_state_dict(401, **SMALL)
    m = make_model(SMALL, 4, 401, device="cuda").eval()
    x0 = torch.tensor(gen.randint(9, (2, 3), 0, 34), device="cuda")
    out = m.generate(x0)
    assert out.shape == (2, 3 + 33)
    # every greedy step picks the oracle's argmax of the last position (cropped context)
    st = {k: torch.tensor(v) for k, v in sd.items()}
    xs = out.cpu()
    for t in range(3, 3 + 33):
        ctx = xs[:, max(0, t - 33):t]
        ref = od.decoder_forward(st, ctx, 4)[:, -1].argmax(-1)
        assert torch.equal(ref, xs[:, t]), t


@pytest.mark.gpu
def test_sequence_longer_than_mask_raises():
    m = make_model(SMALL, 4, 401, device="cuda").eval()
    with pytest.raises(RuntimeError):
        with torch.no_grad():
            m(torch.zeros(1, 40, dtype=torch.long, device="cuda"))


@pytest.fixture
def fp32_mode():
    from arcweld.precision import operands
    with operands(torch.float32):
        yield


@pytest.mark.gpu
@pytest.mark.parametrize("n_head", [4, 2])
def test_kv_cache_prefill_and_decode_match_full_forward(fp32_mode, n_head):
    """forward_cached: the prefill's last-position logits and each cached decode step equal the
    reference's full recompute (forward over the whole prefix) within the fp32 tolerance."""
    from arcweld import decoder as dec
    m = make_model(SMALL, n_head, 401, device="cuda").eval()
    B, T0 = 3, 7
    x = torch.tensor(gen.randint(450, (B, 20), 0, SMALL["n_classes"]), device="cuda")
    cache = dec.KVCache(m, B, SMALL["seq_len"])
    got = dec.forward_cached(m, x[:, :T0], cache, 0)
    with torch.no_grad():
        ref = m(x[:, :T0])[:, -1]
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    for t in range(T0, 20):
        got = dec.forward_cached(m, x[:, t:t + 1], cache, t)
        with torch.no_grad():
            ref = m(x[:, :t + 1])[:, -1]
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4, msg=f"position {t}")


@pytest.mark.gpu
def test_cached_generate_matches_reference_recompute(fp32_mode):
    """generate(use_cache=True) produces the same greedy continuation as the reference's recompute loop,
    including the steps after the context is cropped to seq_len (the cache is re-prefilled there)."""
    m = make_model(SMALL, 4, 403, device="cuda").eval()
    x = torch.tensor(gen.randint(451, (2, 9), 0, SMALL["n_classes"]), device="cuda")
    a = m.generate(x, use_cache=True)
    b = m.generate(x, use_cache=False)
    assert a.shape == (2, 9 + SMALL["seq_len"])
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("task", ["gen", "cls"])
def test_fused_train_step_matches_autograd_and_split_point_is_final(fp32_parity, task):
    """fused_train_step (no autograd; what a captured data-parallel step runs) gives the autograd step's loss and
    gradients, and at its mid_hook every gradient of backward_late_parameters() is final while every other one is
    still untouched -- the invariant the overlapped all-reduce of the later blocks relies on."""
    m = make_model(dict(SMALL, n_blocks=4), 4, 411, device="cuda").train()
    batch = inputs(4, 33, 34, 412, "cuda")
    x, y, cond = batch
    loss_ref, _ = _step(m, task, batch)
    ref = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    names = [n for n, _ in m.named_parameters()]
    params = list(m.parameters())
    late = set(id(p) for p in m.backward_late_parameters())
    snap = []
    loss = m.fused_train_step((x, cond, y), 1.0, mid_hook=lambda: snap.append([p.grad.clone() for p in params]))
    assert len(snap) == 1
    np.testing.assert_allclose(loss.item(), loss_ref.item(), rtol=1e-6)
    for i, (n, p) in enumerate(zip(names, params)):
        if n in ref:
            torch.testing.assert_close(p.grad, ref[n], rtol=1e-5, atol=1e-7, msg=n)
            if id(p) in late:
                assert torch.equal(snap[0][i], p.grad), n
            else:
                assert not snap[0][i].any(), n
        else:
            assert not p.grad.any(), n


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_kv_cache_full_size_decode_matches_full_forward(dtype):
    """The KV-cache path at the full size (d 512, 8 heads of 64, 8 blocks, T 321, V 514): a 300-token prefill,
    then 20 cached decode steps up to position 320, each against the full-recompute forward (fp32: 1e-4; bf16
    operands: the same kernels' bf16 recompute, 2e-2), and greedy generation identical to the recompute loop."""
    from arcweld import decoder as dec
    from arcweld.precision import operands
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    tol = 1e-4 if dtype == "fp32" else 2e-2
    m = make_model(FULL, 8, 405, device="cuda").eval()
    B, T0 = 2, 300
    x = torch.tensor(gen.randint(452, (B, 321), 0, FULL["n_classes"]), device="cuda")
    with operands(dt):
        cache = dec.KVCache(m, B, FULL["seq_len"])
        got = dec.forward_cached(m, x[:, :T0], cache, 0)
        with torch.no_grad():
            ref = m(x[:, :T0])[:, -1]
        torch.testing.assert_close(got, ref, rtol=tol, atol=tol)
        for t in range(T0, 321):
            got = dec.forward_cached(m, x[:, t:t + 1], cache, t)
            if t % 5 == 0 or t == 320:
                with torch.no_grad():
                    ref = m(x[:, :t + 1])[:, -1]
                torch.testing.assert_close(got, ref, rtol=tol, atol=tol, msg=f"position {t}")
    if dtype == "fp32":
        with operands(torch.float32):
            m2 = make_model(dict(FULL, seq_len=24), 8, 405, device="cuda").eval()
            p = torch.tensor(gen.randint(453, (2, 5), 0, FULL["n_classes"]), device="cuda")
            assert torch.equal(m2.generate(p, use_cache=True), m2.generate(p, use_cache=False))
