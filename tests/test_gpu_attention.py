"""Causal attention kernels (aw_attn_fwd / aw_attn_bwd) against a plain torch fp32 reference of
CausalSelfAttention (model/transformer_block.py:37-63, attention dropout 0).  fp32 operands -> the VALU
kernels (tolerance 1e-4); bf16 operands -> the MFMA kernels at head size 64 (VALU otherwise), compared on the
same bf16-rounded inputs with bf16-output tolerance."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def reference(qkv, B, T, nh, d, dy):
    q, k, v = qkv.float().view(B, T, 3 * d).split(d, dim=2)
    hs = d // nh
    q = q.reshape(B, T, nh, hs).transpose(1, 2).requires_grad_()
    k = k.reshape(B, T, nh, hs).transpose(1, 2).requires_grad_()
    v = v.reshape(B, T, nh, hs).transpose(1, 2).requires_grad_()
    att = (q @ k.transpose(-2, -1)) / math.sqrt(hs)
    mask = torch.tril(torch.ones(T, T, device=qkv.device, dtype=torch.bool))
    att = att.masked_fill(~mask, float("-inf"))
    lse = torch.logsumexp(att, dim=-1)
    y = (torch.softmax(att, dim=-1) @ v).transpose(1, 2).reshape(B * T, d)
    y.backward(dy.float())
    dq = q.grad.transpose(1, 2).reshape(B * T, d)
    dk = k.grad.transpose(1, 2).reshape(B * T, d)
    dv = v.grad.transpose(1, 2).reshape(B * T, d)
    return y.detach(), lse.detach().reshape(-1), torch.cat([dq, dk, dv], dim=1)


def run(qkv, B, T, nh, d, dy):
    from arcweld import kernels as K
    R = B * T
    y = torch.empty(R, d, device="cuda", dtype=qkv.dtype)
    lse = torch.empty(B * nh * T, device="cuda")
    K.attn_fwd(qkv, B, T, nh, d, y, lse)
    dqkv = torch.empty(R, 3 * d, device="cuda", dtype=qkv.dtype)
    ws = torch.empty(B * nh * T, device="cuda")
    K.attn_bwd(qkv, y, dy, lse, B, T, nh, d, dqkv, ws)
    return y, lse, dqkv


def _inputs(B, T, d, dtype, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    qkv = torch.randn(B * T, 3 * d, device="cuda", generator=g).to(dtype)
    dy = torch.randn(B * T, d, device="cuda", generator=g).to(dtype)
    return qkv, dy


@pytest.mark.parametrize("T", [1, 33, 64, 65, 128, 200, 321])
@pytest.mark.parametrize("hs", [16, 64])
def test_attention_fp32(T, hs):
    B, nh = 2, 2
    d = hs * nh
    qkv, dy = _inputs(B, T, d, torch.float32, T + hs)
    y, lse, dqkv = run(qkv, B, T, nh, d, dy)
    ry, rl, rg = reference(qkv, B, T, nh, d, dy)
    torch.testing.assert_close(y, ry, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lse, rl, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dqkv, rg, rtol=1e-4, atol=2e-4)


@pytest.mark.parametrize("T", [1, 17, 64, 65, 96, 97, 127, 128, 129, 200, 257, 300, 321, 384, 385])
@pytest.mark.parametrize("hs,nh", [(64, 2), (64, 8), (32, 4)])
def test_attention_bf16(T, hs, nh):
    B = 3
    d = hs * nh
    qkv, dy = _inputs(B, T, d, torch.bfloat16, 7 * T + hs)
    y, lse, dqkv = run(qkv, B, T, nh, d, dy)
    ry, rl, rg = reference(qkv, B, T, nh, d, dy)
    torch.testing.assert_close(y.float(), ry, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, rl, rtol=1e-3, atol=1e-3)
    err = (dqkv.float() - rg).abs().max().item()
    assert err <= 3e-2 * rg.abs().max().item() + 2e-2, err
    # relative Frobenius error of each of dq, dk, dv
    for j in range(3):
        a, r = dqkv.float()[:, j * d:(j + 1) * d], rg[:, j * d:(j + 1) * d]
        assert (a - r).norm().item() <= 1e-2 * r.norm().item() + 1e-4, j   # dq is exactly 0 at T = 1


@pytest.mark.parametrize("R", [5, 1000, 5000, 16371])
@pytest.mark.parametrize("D", [64, 512, 1024])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_bwd(R, D, out_dtype):
    """aw_layernorm_fwd / aw_layernorm_bwd (vectorised at D % 256 == 0) vs torch layer_norm in fp32, including
    the accumulate-into-dx form and the dropout-masked operand copy dx2 (regenerated mask).  R = 5000 and 16371
    (the decoder's 51 x 321 rows) exceed the backward's 2048 waves, so each wave walks several rows (the next-row
    prefetch path); R = 5 leaves most waves without a row."""
    from arcweld import kernels as K
    g = torch.Generator(device="cuda").manual_seed(D)
    x = torch.randn(R, D, device="cuda", generator=g) * 3 + 1
    w = torch.randn(D, device="cuda", generator=g)
    b = torch.randn(D, device="cuda", generator=g)
    dy = torch.randn(R, D, device="cuda", generator=g)
    y = torch.empty(R, D, device="cuda", dtype=out_dtype)
    mu, rs = torch.empty(R, device="cuda"), torch.empty(R, device="cuda")
    K.layernorm_fwd(x, w, b, 1e-5, y, mu, rs)
    xr = x.clone().requires_grad_()
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    ry = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-5)
    tol = 1e-5 if out_dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.float(), ry.detach(), rtol=tol, atol=tol)
    ry.backward(dy)
    prior = torch.randn(R, D, device="cuda", generator=g)
    dx = prior.clone()
    dw, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    dx2 = torch.empty(R, D, device="cuda", dtype=out_dtype)
    K.layernorm_bwd(x, dy, w, mu, rs, dx, True, dw, db, dx2=dx2, drop=(0.25, 1234))
    torch.testing.assert_close(dx, prior + xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw, wr.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    kept = dx2.float() != 0
    frac = kept.float().mean().item()
    assert abs(frac - 0.75) < max(0.03, 4 * (0.1875 / kept.numel()) ** 0.5), frac   # 4 sigma at small R
    torch.testing.assert_close(dx2.float()[kept], (dx / 0.75)[kept], rtol=tol, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("hs,T", [(8, 17), (12, 33), (24, 70), (40, 65), (6, 5)])
def test_attention_any_head_size_fp32(hs, T):
    """Head sizes outside 16/32/64/128 (the reference allows any d_model % n_head == 0) run the runtime-size
    kernels: forward and every input gradient against the torch fp32 reference."""
    from arcweld import kernels as K
    torch.manual_seed(hs * 100 + T)
    B, nh = 2, 3
    d = nh * hs
    qkv = torch.randn(B * T, 3 * d, device="cuda")
    y, lse = torch.empty(B * T, d, device="cuda"), torch.empty(B * nh * T, device="cuda")
    K.attn_fwd(qkv, B, T, nh, d, y, lse)
    dy = torch.randn(B * T, d, device="cuda")
    dqkv, ws = torch.empty_like(qkv), torch.empty(B * nh * T, device="cuda")
    K.attn_bwd(qkv, y, dy, lse, B, T, nh, d, dqkv, ws)
    ref_in = qkv.detach().clone().requires_grad_(True)
    q, k, v = ref_in.view(B, T, 3 * d).split(d, dim=2)
    q, k, v = (t.reshape(B, T, nh, hs).transpose(1, 2) for t in (q, k, v))
    att = (q @ k.transpose(-2, -1)) / math.sqrt(hs)
    att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device="cuda").tril(), float("-inf")).softmax(-1)
    ref = (att @ v).transpose(1, 2).reshape(B * T, d)
    ref.backward(dy)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dqkv, ref_in.grad, rtol=1e-4, atol=1e-4)


def _dropout_keep(seed, B, nh, T, p):
    """The kernels' counter-based mask (common.h aw_hash_group / aw_dropout_scale), restated in numpy: element
    e = ((b*nh + h)*T + i)*T + j is dropped iff its 16-bit slice of splitmix64(seed, e >> 2) < round(p * 65536)."""
    import numpy as np
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    e = np.arange(B * nh * T * T, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (e // np.uint64(4) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> (np.uint64(16) * (e & np.uint64(3)))) & np.uint64(0xFFFF)
    keep = u >= np.uint64(int(p * 65536 + 0.5))
    del M
    return torch.tensor(keep.reshape(B, nh, T, T))


@pytest.mark.gpu
@pytest.mark.parametrize("hs,T,dtype", [(16, 40, torch.float32), (64, 70, torch.float32), (64, 45, torch.bfloat16),
                                        (12, 33, torch.float32)])
def test_attention_probability_dropout_fp32(hs, T, dtype):
    """att_dropout > 0 (model/transformer_block.py:44-57): the kernels' output and input gradients equal torch's
    attention with the same mask (regenerated here from the counter hash) applied after the softmax and 1/(1-p)
    scaling."""
    from arcweld import kernels as K
    torch.manual_seed(hs + T)
    B, nh, p, seed = 2, 2, 0.2, 12345
    d = nh * hs
    qkv = torch.randn(B * T, 3 * d, device="cuda").to(dtype)
    y, lse = torch.empty(B * T, d, device="cuda", dtype=dtype), torch.empty(B * nh * T, device="cuda")
    K.attn_fwd(qkv, B, T, nh, d, y, lse, drop=(p, seed))
    dy = torch.randn(B * T, d, device="cuda").to(dtype)
    dqkv, ws = torch.empty_like(qkv), torch.empty(B * nh * T, device="cuda")
    K.attn_bwd(qkv, y, dy, lse, B, T, nh, d, dqkv, ws, drop=(p, seed))
    keep = _dropout_keep(seed, B, nh, T, p).cuda()
    assert 0.7 < keep.float().mean().item() < 0.9
    ref_in = qkv.float().detach().clone().requires_grad_(True)
    q, k, v = ref_in.view(B, T, 3 * d).split(d, dim=2)
    q, k, v = (t.reshape(B, T, nh, hs).transpose(1, 2) for t in (q, k, v))
    att = (q @ k.transpose(-2, -1)) / math.sqrt(hs)
    att = att.masked_fill(~torch.ones(T, T, dtype=torch.bool, device="cuda").tril(), float("-inf")).softmax(-1)
    att = att * keep / (1 - p)
    ref = (att @ v).transpose(1, 2).reshape(B * T, d)
    ref.backward(dy.float())
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(y.float(), ref.detach(), rtol=tol, atol=tol)
    torch.testing.assert_close(dqkv.float(), ref_in.grad, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_decoder_trains_with_attention_dropout():
    """MyTransformerDecoder(att_dropout > 0) trains through the fused path: the masks change per step (device
    counter), eval mode is deterministic and equals the att_dropout = 0 model."""
    from arcweld.precision import operands
    from model.transformer_decoder import MyTransformerDecoder
    with operands(torch.float32):
        torch.manual_seed(0)
        m = MyTransformerDecoder(d_model=64, n_classes=34, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0,
                                 att_dropout=0.3).cuda().train()
        x = torch.randint(0, 34, (3, 33), device="cuda")
        a = m(x)
        b = m(x)
        assert not torch.equal(a, b)
        a.sum().backward()
        assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
        m.eval()
        ref = MyTransformerDecoder(d_model=64, n_classes=34, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0,
                                   att_dropout=0.0).cuda().eval()
        ref.load_state_dict(m.state_dict())
        with torch.no_grad():
            torch.testing.assert_close(m(x), ref(x), rtol=0, atol=0)
