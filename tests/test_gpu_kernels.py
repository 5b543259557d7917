"""Kernel-level parity on the MI355X: every GEMM form / epilogue against a plain PyTorch fp32 reference of the
same op, and the VQ kernel against the reference's own golden indices (bit-exact) and the CPU oracle."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import gen
from oracle import vqvae as ov

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def K():
    from arcweld import kernels
    return kernels


@pytest.fixture(params=[0, 256], ids=["tile_auto", "tile256"])
def tile(request, K):
    """Runs a test under the automatic tile policy and with every eligible (bf16, non-ragged) launch forced onto
    the 256x128 three-stage pipeline (aw_gemm_set_tile), so both kernels are covered at small shapes."""
    from arcweld import _native
    _native.call("aw_gemm_set_tile", request.param)
    yield request.param
    _native.call("aw_gemm_set_tile", 0)


def _rand(shape, seed, dtype=torch.float32, scale=1.0):
    return torch.tensor(gen.normal(seed, shape, scale)).to(DEV, dtype)


def _tol(dtype, K):
    return (2e-5 * np.sqrt(K / 64), 1e-5) if dtype == torch.float32 else (2e-2, 1e-2)


def _padded(rows, cols, seed, dtype):
    """(rows, cols) view of a (rows, roundup(cols, 8)) buffer: 16-B aligned rows, ragged logical width."""
    ld = (cols + 7) // 8 * 8
    return _rand((rows, ld), seed, dtype)[:, :cols]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("a_trans,b_trans", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,Kd", [(256, 128, 64), (300, 200, 72), (17, 514, 512), (1000, 64, 48), (64, 96, 514)])
def test_gemm_layouts(K, tile, dtype, a_trans, b_trans, M, N, Kd):
    A = _padded(Kd, M, 1, dtype) if a_trans else _padded(M, Kd, 1, dtype)
    B = _padded(Kd, N, 2, dtype) if b_trans else _padded(N, Kd, 2, dtype)
    C = torch.empty(M, N, device=DEV)
    K.gemm(A, B, M, N, Kd, a_trans=a_trans, b_trans=b_trans, C=C)
    Af = A.float().cpu()
    Bf = B.float().cpu()
    ref = (Af.t() if a_trans else Af) @ (Bf if b_trans else Bf.t())
    rtol, atol = _tol(dtype, Kd)
    torch.testing.assert_close(C.cpu(), ref, rtol=rtol, atol=atol * np.sqrt(Kd))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_chain(K, tile, dtype):
    M, N, Kd = 384, 256, 128
    A = _rand((M, Kd), 3, dtype)
    W = _rand((N, Kd), 4, dtype, 0.1)
    bias = _rand((N,), 5)
    pre = _rand((M, N), 6)
    resid = _rand((M, N), 7)
    C = torch.empty(M, N, device=DEV)
    C2 = torch.empty(M, N, device=DEV, dtype=dtype)
    stats = torch.zeros(2 * 64, device=DEV, dtype=torch.float64)
    rows = torch.zeros(M, device=DEV)
    K.gemm(A, W, M, N, Kd, C=C, C2=C2, c2_mode=1, bias=bias, pre=pre, resid=resid, colstats=stats, stats_mod=64,
           a_rowsum=rows)
    acc = A.float().cpu() @ W.float().cpu().t()
    pre_c = pre.cpu()
    gp = 0.5 * (1 + torch.erf(pre_c / np.sqrt(2))) + pre_c * torch.exp(-0.5 * pre_c ** 2) / np.sqrt(2 * np.pi)
    v = (acc + bias.cpu()) * gp + resid.cpu()
    rtol, atol = _tol(dtype, Kd)
    torch.testing.assert_close(C.cpu(), v, rtol=rtol, atol=atol * 10)
    torch.testing.assert_close(C2.float().cpu(), F.gelu(v), rtol=2e-2 if dtype != torch.float32 else 1e-5,
                               atol=atol * 10)
    st = stats.cpu()
    vv = C.cpu().double()
    # fp32 per-wave partials, f64 across waves
    torch.testing.assert_close(st[:64], vv.view(M, N // 64, 64).sum((0, 1)), rtol=2e-5, atol=1e-3)
    torch.testing.assert_close(st[64:], (vv ** 2).view(M, N // 64, 64).sum((0, 1)), rtol=2e-5, atol=1e-3)
    torch.testing.assert_close(rows.cpu(), A.float().cpu().sum(1), rtol=1e-5, atol=1e-4)


def test_gemm_beta_and_dropout(K, tile):
    M, N, Kd = 256, 128, 64
    A = _rand((M, Kd), 8)
    W = _rand((N, Kd), 9)
    C = _rand((M, N), 10)
    C0 = C.cpu().clone()
    K.gemm(A, W, M, N, Kd, C=C, beta=1.0, alpha=0.5)
    torch.testing.assert_close(C.cpu(), C0 + 0.5 * (A.cpu() @ W.cpu().t()), rtol=1e-5, atol=1e-4)
    D = torch.empty(M, N, device=DEV)
    K.gemm(A, W, M, N, Kd, C=D, drop=(0.25, 1234))
    ref = A.cpu() @ W.cpu().t()
    d = D.cpu()
    zero = d == 0
    assert 0.2 < zero.float().mean().item() < 0.3
    torch.testing.assert_close(d[~zero], ref[~zero] / 0.75, rtol=1e-5, atol=1e-4)
    D2 = torch.empty(M, N, device=DEV)
    K.gemm(A, W, M, N, Kd, C=D2, drop=(0.25, 1234))
    assert torch.equal(D.cpu(), D2.cpu())          # counter-based mask: reproducible for the backward


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_implicit_conv3(K, tile, dtype):
    """Decoder conv (k=3, pad=1 per window of S tokens): forward, input-gradient and weight-gradient forms."""
    Bw, S, Cin, Cout = 6, 16, 64, 128
    M = Bw * S
    x = _rand((M, Cin), 11, dtype)
    W = torch.tensor(gen.normal(12, (Cout, Cin, 3), 0.1))
    dev_dtype = dtype
    Wk = torch.empty(Cout, 3 * Cin, device=DEV, dtype=dev_dtype)
    K.weight_relayout(W.to(DEV), Cout, Cin, 3, 0, 1, Wk)
    y = torch.empty(M, Cout, device=DEV)
    K.gemm(x, Wk, M, Cout, 3 * Cin, conv=(Cin, S, 1, 0), C=y)
    xr = x.float().cpu().view(Bw, S, Cin).transpose(1, 2)
    Wr = W.to(dtype).float()
    ref = F.conv1d(xr, Wr, padding=1).transpose(1, 2).reshape(M, Cout)
    rtol, atol = _tol(dtype, 3 * Cin)
    torch.testing.assert_close(y.cpu(), ref, rtol=rtol, atol=atol * 10)
    # input gradient: g_in = conv_transpose of g_out
    g = _rand((M, Cout), 13, dtype)
    Wd = torch.empty(3 * Cout, Cin, device=DEV, dtype=dev_dtype)
    K.weight_relayout(W.to(DEV), Cout, Cin, 3, 0, 2, Wd)
    gin = torch.empty(M, Cin, device=DEV)
    K.gemm(g, Wd, M, Cin, 3 * Cout, b_trans=True, conv=(Cout, S, -1, 0), C=gin)
    xr2 = xr.clone().requires_grad_(True)
    out = F.conv1d(xr2, Wr.clone().requires_grad_(True), padding=1)
    gr = g.float().cpu().view(Bw, S, Cout).transpose(1, 2)
    out.backward(gr)
    torch.testing.assert_close(gin.cpu(), xr2.grad.transpose(1, 2).reshape(M, Cin), rtol=rtol, atol=atol * 10)
    # weight gradient: dWk[o][(j,i)] = sum_m g[m][o] x[m+j-1][i]
    dWk = torch.empty(Cout, 3 * Cin, device=DEV)
    K.gemm(g, x, Cout, 3 * Cin, M, a_trans=True, b_trans=True, conv=(Cin, S, 1, 1), C=dWk)
    G = torch.zeros(Cout, Cin, 3, device=DEV)
    K.weight_grad_scatter(dWk, Cout, Cin, 3, 0, 1, G)
    Wg = Wr.clone().requires_grad_(True)
    F.conv1d(xr, Wg, padding=1).backward(gr)
    torch.testing.assert_close(G.cpu(), Wg.grad, rtol=rtol, atol=atol * 30)


@pytest.mark.parametrize("conv", [False, True], ids=["plain", "conv3"])
@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_gemm_bf16_residual_stream_epilogues(K, tile, conv, p_drop):
    """The bf16-mode ResBlock residual launches with bf16 residual streams (aw_gemm_args.resid_dtype; arcweld/vqvae.py
    resid_dtype): forward  y = x + drop(A.W^T + b) -> C (bf16) and GELU(y) (bf16);  input gradient
    gx' = gx + (g.W) * GELU'(x) -> C (bf16) with the dropout-masked / plain bf16 copy; and the first gradient launch
    C (bf16) + masked copy.  Each against the same launch with an f32 residual stream (bit-identical f32 math, so the
    bf16 outputs equal the f32 outputs rounded) and against torch fp32 at p = 0."""
    bf = torch.bfloat16
    Bw, S, Cin, Cout = 16, 16, 128, 128
    M = Bw * S
    cv = (Cin, S, 1, 0) if conv else None
    Kd = 3 * Cin if conv else Cin
    A = _rand((M, Cin), 61, bf)
    W = _rand((Cout, Kd), 62, bf, 0.05)
    bias = _rand((Cout,), 63)
    x = _rand((M, Cout), 64, bf)
    outs = {}
    for rdt in (torch.float32, bf):
        C = torch.empty(M, Cout, device=DEV, dtype=rdt)
        C2 = torch.empty(M, Cout, device=DEV, dtype=bf)
        K.gemm(A, W, M, Cout, Kd, conv=cv, bias=bias, drop=(p_drop, 77), resid=x.to(rdt), C=C, C2=C2, c2_mode=1)
        outs[rdt] = (C, C2)
    torch.testing.assert_close(outs[bf][0], outs[torch.float32][0].to(bf), rtol=0, atol=0)
    torch.testing.assert_close(outs[bf][1], outs[torch.float32][1], rtol=0, atol=0)
    if p_drop == 0.0:
        if conv:
            xr = A.float().cpu().view(Bw, S, Cin).transpose(1, 2)
            Wr = W.float().cpu().view(Cout, 3, Cin).permute(0, 2, 1)
            acc = F.conv1d(xr, Wr, padding=1).transpose(1, 2).reshape(M, Cout)
        else:
            acc = A.float().cpu() @ W.float().cpu().t()
        v = acc + bias.cpu() + x.float().cpu()
        torch.testing.assert_close(outs[bf][0].float().cpu(), v, rtol=8e-3, atol=2e-2)
    # input gradient: C = gx + (g . W) * GELU'(x), C2 = masked (drop2) or plain copy
    Wd = _rand((Cout if not conv else 3 * Cout, Cin), 66, bf, 0.05)
    gx = _rand((M, Cin), 67, bf)
    pre = _rand((M, Cin), 68, bf)
    dcv = (Cout, S, -1, 0) if conv else None
    Kb = 3 * Cout if conv else Cout
    g = _rand((M, Cout), 65, bf)
    for mode in (2, 3):
        res = {}
        for rdt in (torch.float32, bf):
            C = torch.empty(M, Cin, device=DEV, dtype=rdt)
            C2 = torch.empty(M, Cin, device=DEV, dtype=bf)
            K.gemm(g, Wd, M, Cin, Kb, b_trans=True, conv=dcv, pre=pre.to(rdt), resid=gx.to(rdt), C=C, C2=C2,
                   c2_mode=mode, drop2=(p_drop, 78))
            res[rdt] = (C, C2)
        torch.testing.assert_close(res[bf][0], res[torch.float32][0].to(bf), rtol=0, atol=0)
        torch.testing.assert_close(res[bf][1], res[torch.float32][1], rtol=0, atol=0)
    if not conv:
        # the first gradient launch of a stack: C (bf16) + masked copy, no residual
        res = {}
        for rdt in (torch.float32, bf):
            C = torch.empty(M, Cin, device=DEV, dtype=rdt)
            C2 = torch.empty(M, Cin, device=DEV, dtype=bf)
            K.gemm(g, Wd, M, Cin, Kb, b_trans=True, C=C, C2=C2, c2_mode=3, drop2=(p_drop, 79))
            res[rdt] = (C, C2)
        torch.testing.assert_close(res[bf][0], res[torch.float32][0].to(bf), rtol=0, atol=0)
        torch.testing.assert_close(res[bf][1], res[torch.float32][1], rtol=0, atol=0)


@pytest.mark.parametrize("tag,Kc,D,N,eseed,estd", [
    ("K512_D64_init", 512, 64, 16384, 201, None),
    ("K512_D64_trained", 512, 64, 16384, 202, 0.08),
    ("K8192_D256_trained", 8192, 256, 4096, 203, 0.05),
])
def test_vq_indices_bit_exact_vs_reference(K, tag, Kc, D, N, eseed, estd):
    g = golden("vq_idx.npz")
    z = gen.normal(210 + Kc, (N, D), 0.08)
    E = gen.uniform(eseed, (Kc, D), -1.0 / Kc, 1.0 / Kc) if estd is None else gen.normal(eseed, (Kc, D), estd)
    zd, Ed = torch.tensor(z, device=DEV), torch.tensor(E, device=DEV)
    zq = torch.empty_like(zd)
    idx = torch.empty(N, dtype=torch.int64, device=DEV)
    counts = torch.zeros(Kc, device=DEV)
    sq = torch.zeros(1, dtype=torch.float64, device=DEV)
    K.vq_forward(zd, Ed, zq, idx, counts, sq)
    ref = g[f"idx_{tag}"].astype(np.int64)
    got = idx.cpu().numpy()
    gap = g[f"gap_{tag}"]
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, f"{bad.size} index mismatches; top-2 gaps there: {gap[bad][:8]}"
    out2 = torch.empty(2, device=DEV)
    K.vq_finalize(counts, sq, N, Kc, D, 0.25, out2[0:1], out2[1:2])
    np.testing.assert_allclose(out2[0].item(), g[f"loss_{tag}"], rtol=1e-5)
    np.testing.assert_allclose(out2[1].item(), g[f"perplexity_{tag}"], rtol=1e-5)
    np.testing.assert_array_equal(counts.cpu().numpy(), np.bincount(ref, minlength=Kc).astype(np.float32))


def test_vq_small_forward_backward_vs_reference(K):
    g = golden("vq_small.npz")
    E = torch.tensor(gen.uniform(101, (64, 16), -0.5, 0.5), device=DEV)
    z = torch.tensor(gen.normal(102, (16 * 16, 16), 0.5), device=DEV)
    g_zq = torch.tensor(gen.normal(103, (16 * 16, 16), 1.0), device=DEV)
    N = z.shape[0]
    zq = torch.empty_like(z)
    idx = torch.empty(N, dtype=torch.int64, device=DEV)
    counts = torch.zeros(64, device=DEV)
    sq = torch.zeros(1, dtype=torch.float64, device=DEV)
    K.vq_forward(z, E, zq, idx, counts, sq)
    out2 = torch.empty(2, device=DEV)
    K.vq_finalize(counts, sq, N, 64, 16, 0.25, out2[0:1], out2[1:2])
    assert np.array_equal(idx.cpu().numpy(), g["idx"].reshape(-1))
    np.testing.assert_allclose(zq.cpu().numpy().reshape(g["z_q"].shape), g["z_q"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(out2[0].item(), g["loss"], rtol=1e-6)
    np.testing.assert_allclose(out2[1].item(), g["perplexity"], rtol=1e-6)
    dz = torch.empty_like(z)
    dE = torch.zeros_like(E)
    gl = torch.tensor([float(g["g_loss"])], device=DEV)
    K.vq_backward(z, E, idx, g_zq, gl, 0.25, dz, dE)
    np.testing.assert_allclose(dz.cpu().numpy().reshape(g["dz"].shape), g["dz"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(dE.cpu().numpy(), g["dE"], rtol=1e-4, atol=1e-7)
    oh = torch.empty(N, 64, device=DEV)
    K.vq_onehot(idx, 64, oh)
    np.testing.assert_array_equal(oh.cpu().numpy().argmax(1), g["idx"].reshape(-1))
    assert oh.sum().item() == N


@pytest.mark.parametrize("cdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Kc,D,N", [(512, 64, 16384), (64, 16, 1000)])
def test_vq_operand_copies_match_the_cast_outputs(K, cdt, Kc, D, N):
    """aw_vq_forward_ex / aw_vq_backward_ex: the operand copies are exactly the cast of z_q and dz (the step's cast
    launches they replace), and the primary outputs are unchanged by writing them."""
    z = torch.tensor(gen.normal(301, (N, D), 0.08), device=DEV)
    E = torch.tensor(gen.normal(302, (Kc, D), 0.08), device=DEV)
    outs = []
    for copy in (False, True):
        zq, idx = torch.empty_like(z), torch.empty(N, dtype=torch.int64, device=DEV)
        counts, sq = torch.zeros(Kc, device=DEV), torch.zeros(1, dtype=torch.float64, device=DEV)
        zc = torch.full((N, D), float("nan"), device=DEV, dtype=cdt) if copy else None
        K.vq_forward(z, E, zq, idx, counts, sq, zq_copy=zc)
        g_zq = torch.tensor(gen.normal(303, (N, D), 1.0), device=DEV)
        dz, dE = torch.empty_like(z), torch.zeros_like(E)
        dc = torch.full((N, D), float("nan"), device=DEV, dtype=cdt) if copy else None
        K.vq_backward(z, E, idx, g_zq, torch.tensor([1.5], device=DEV), 0.25, dz, dE, dz_copy=dc)
        outs.append((zq, idx, counts, sq, dz, dE))
        if copy:
            assert torch.equal(zc, zq.to(cdt))
            assert torch.equal(dc, dz.to(cdt))
    for i, (a, b) in enumerate(zip(*outs)):
        if i in (3, 5):   # sqerr (f64) and dE (f32): atomics, summation order differs run to run
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9)
        else:
            assert torch.equal(a, b)


@pytest.mark.parametrize("Kc,D,N", [(512, 64, 16384), (512, 64, 1000), (64, 16, 1000), (8192, 256, 4096)])
@pytest.mark.parametrize("G", [2, 8])
def test_vq_grouped_counts_sum_to_the_counts(K, Kc, D, N, G):
    """aw_vq_forward_ex2 / aw_vq_finalize_ex: the count_groups partial histograms sum exactly to the count_groups 1
    counts (both kernels: pinned MFMA at K <= 512, streaming VALU above), every other output is unchanged, and the
    finalize over the partials gives the same loss and perplexity bits."""
    z = torch.tensor(gen.normal(311, (N, D), 0.08), device=DEV)
    E = torch.tensor(gen.normal(312, (Kc, D), 0.08), device=DEV)
    outs = []
    for cg in (1, G):
        zq, idx = torch.empty_like(z), torch.empty(N, dtype=torch.int64, device=DEV)
        counts, sq = torch.zeros(cg * Kc, device=DEV), torch.zeros(1, dtype=torch.float64, device=DEV)
        K.vq_forward(z, E, zq, idx, counts, sq, count_groups=cg)
        fin = torch.empty(2, device=DEV)
        K.vq_finalize(counts, sq, N, Kc, D, 0.25, fin[0:1], fin[1:2], count_groups=cg)
        outs.append((zq, idx, counts.view(cg, Kc).sum(0), fin))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])
    assert torch.equal(outs[0][2], torch.bincount(outs[0][1], minlength=Kc).float())
    torch.testing.assert_close(outs[0][3], outs[1][3], rtol=1e-6, atol=0)   # sqerr: f64 atomics, order varies


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("use_ws", [True, False])
def test_gemm_split_k_accumulate_colmap(K, tile, dtype, use_ws):
    """Weight-gradient form (A^T B, long K): split-K through slabs (workspace) or atomics, accumulated into a
    strided reference layout via the column map (conv weight (O, I, 3): colmap(c) = (c % I)*3 + c // I)."""
    import ctypes
    from arcweld import _native as nat
    M, I, Kd = 192, 96, 4096
    N = 3 * I
    A = _rand((Kd, M), 21, dtype)
    B = _rand((Kd, N), 22, dtype)
    G0 = _rand((M, I, 3), 23)
    G = G0.clone()
    if use_ws:
        K.gemm(A, B, M, N, Kd, a_trans=True, b_trans=True, C=G.view(M, 3 * I), accumulate=True, col_map=(I, 3, 0))
    else:  # force the atomic path: call the plain entry point (no workspace)
        a = nat.GemmArgs()
        a.M, a.N, a.K, a.a_dtype = M, N, Kd, nat.dtype_code(dtype)
        a.A, a.lda, a.a_trans = A.data_ptr(), M, 1
        a.B, a.ldb, a.b_trans = B.data_ptr(), N, 1
        a.alpha = 1.0
        a.C, a.ldc, a.c_dtype = G.data_ptr(), 3 * I, 0
        a.accumulate, a.col_mod, a.col_mul, a.col_off = 1, I, 3, 0
        nat.call("aw_gemm", ctypes.byref(a), torch.cuda.current_stream().cuda_stream)
    prod = (A.float().cpu().t() @ B.float().cpu()).view(M, 3, I).permute(0, 2, 1)   # [o][i][j]
    ref = G0.cpu() + prod
    rtol, atol = _tol(dtype, Kd)
    torch.testing.assert_close(G.cpu(), ref, rtol=rtol, atol=atol * np.sqrt(Kd) * 4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("conv", [False, True])
def test_gemm_grouped_weight_grads_match_single_launches(K, tile, dtype, conv):
    """aw_gemm_grouped (deferred ResBlock weight gradients, one launch for the stack) == one aw_gemm per problem:
    accumulate mode with the conv-tap column map, fused bias-gradient row sums, per-group pointers."""
    S, Cin, Cout, Ntok = 16, 64, 128, 16 * 40
    probs_g, probs_s, outs_g, outs_s = [], [], [], []
    for g in range(3):
        go = _rand((Ntok, Cout), 30 + g, dtype)
        x = _rand((Ntok, Cin), 40 + g, dtype)
        for outs, probs in ((outs_g, probs_g), (outs_s, probs_s)):
            Wg = torch.zeros(Cout, Cin, 3, device=DEV)
            bg = torch.zeros(Cout, device=DEV)
            outs.append((Wg, bg))
            if conv:
                kw = dict(a_trans=True, b_trans=True, conv=(Cin, S, 1, 1), C=Wg.view(Cout, 3 * Cin), accumulate=True,
                          col_map=(Cin, 3, 0), a_rowsum=bg)
                probs.append((go, x, Cout, 3 * Cin, Ntok, kw))
            else:
                kw = dict(a_trans=True, b_trans=True, C=Wg.view(Cout, 3 * Cin), accumulate=True, col_map=(0, 3, 1),
                          a_rowsum=bg)
                probs.append((go, x, Cout, Cin, Ntok, kw))
    K.gemm_grouped(probs_g)
    for (A, B, M, N, Kd, kw) in probs_s:
        K.gemm(A, B, M, N, Kd, **kw)
    rtol, atol = _tol(dtype, Ntok)
    for (Wg, bg), (Ws, bs) in zip(outs_g, outs_s):
        assert Wg.abs().sum() > 0
        torch.testing.assert_close(Wg.cpu(), Ws.cpu(), rtol=rtol, atol=atol * 10)
        torch.testing.assert_close(bg.cpu(), bs.cpu(), rtol=1e-5, atol=1e-4)


def _shift_taps(x, S):
    """[tokens][cin] -> [tokens][3 cin]: tap j holds x[t + j - 1] inside each window of S tokens (zero across)."""
    n, c = x.shape
    w = x.view(n // S, S, c)
    z = torch.zeros_like(w[:, :1])
    prev = torch.cat([z, w[:, :-1]], 1)
    nxt = torch.cat([w[:, 1:], z], 1)
    return torch.cat([prev, w, nxt], 2).view(n, 3 * c)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("conv,G,Cout,Cin,Ntok,S", [(True, 4, 512, 512, 16 * 256, 16), (False, 3, 320, 256, 16 * 300, 16),
                                                    (True, 2, 256, 128, 16 * 40, 16), (True, 3, 200, 192, 40 * 21, 40),
                                                    (True, 2, 136, 64, 8 * 77, 8)])
def test_gemm_grouped_wgrad_tiles_vs_fp32_reference(dtype, conv, G, Cout, Cin, Ntok, S):
    """aw_gemm_grouped at weight-gradient shapes against A^T B in fp32 on the same operands: contiguous rows (the
    optimizer's tap-major decoder weights), the implicit k = 3 taps, ragged M, split token reductions meeting in the
    accumulating atomics, bias row sums, accumulation into a non-zero C; windows of 8, 16 and 40 tokens, ragged M
    and token counts that are not whole 64-token steps (the bf16 conv forms run the three-tap tile)."""
    from arcweld import kernels as K
    N = 3 * Cin if conv else Cin
    probs, refs = [], []
    for g in range(G):
        A = _rand((Ntok, Cout), 60 + g, dtype)
        x = _rand((Ntok, Cin), 70 + g, dtype)
        C0 = _rand((Cout, N), 80 + g)
        b0 = _rand((Cout,), 90 + g)
        C, b = C0.clone(), b0.clone()
        kw = dict(a_trans=True, b_trans=True, C=C, accumulate=True, a_rowsum=b)
        if conv:
            kw["conv"] = (Cin, S, 1, 1)
        probs.append((A, x, Cout, N, Ntok, kw))
        Bf = _shift_taps(x.float(), S) if conv else x.float()
        refs.append((C, b, C0 + A.float().t() @ Bf, b0 + A.float().sum(0)))
    K.gemm_grouped(probs)
    rtol, atol = _tol(dtype, Ntok)
    for C, b, Cr, br in refs:
        torch.testing.assert_close(C, Cr, rtol=rtol, atol=atol * np.sqrt(Ntok) * 4)
        torch.testing.assert_close(b, br, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("act", [0, 1])
def test_gemm_bf16_pre_activation_operand(K, tile, act):
    """pre (the saved GELU pre-activation) may be bf16: identical to passing the same values as f32."""
    M, N, Kd = 256, 256, 128
    A = _rand((M, Kd), 50, torch.bfloat16)
    W = _rand((N, Kd), 51, torch.bfloat16, 0.1)
    pre = _rand((M, N), 52).to(torch.bfloat16)
    resid = _rand((M, N), 53)
    act_code = K.AW_ACT_GELU_TANH if act else K.AW_ACT_GELU_ERF
    outs = []
    for p in (pre, pre.float()):
        C = torch.empty(M, N, device=DEV)
        C2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        K.gemm(A, W, M, N, Kd, b_trans=False, act=act_code, pre=p, resid=resid, C=C, C2=C2, c2_mode=2)
        outs.append((C.cpu(), C2.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("n,off", [(409600, 0), (1001, 0), (4099, 1)])
def test_mse_loss_vs_fp64(K, n, off):
    """aw_mse_fwd / aw_mse_finalize: float4 path, scalar tail, and an unaligned view (scalar path throughout)."""
    from arcweld.functional import mse_loss
    a = torch.tensor(gen.normal(401, (n + off,), 1.0), device=DEV)[off:]
    b = torch.tensor(gen.normal(402, (n + off,), 1.0), device=DEV)[off:]
    got = mse_loss(a, b).item()
    ref = ((a.double() - b.double()) ** 2).mean().item()
    np.testing.assert_allclose(got, ref, rtol=2e-6)


def test_mse_finalize_add_and_counter_zero(K):
    """aw_mse_finalize_add (recon = sq / n, loss = recon + embedding loss in one launch) and
    aw_counter_add_snapshot_zero (dropout counter advance + snapshot + accumulator-block zeroing in one launch)."""
    sq = torch.tensor([1234.5], device=DEV, dtype=torch.float64)
    emb = torch.tensor([0.25], device=DEV)
    recon, loss = torch.empty((), device=DEV), torch.empty((), device=DEV)
    K.mse_finalize_add(sq, 1000, emb, recon, loss)
    assert recon.item() == np.float32(1234.5 / 1000)
    assert loss.item() == np.float32(np.float32(1234.5 / 1000) + np.float32(0.25))
    for nz in (0, 1, 2306, 70001):     # the bench's block (K 512, H 512) and a multi-workgroup block
        ctr = torch.tensor([41], device=DEV, dtype=torch.int64)
        snap = torch.empty(1, device=DEV, dtype=torch.int64)
        z = torch.full((nz + 3,), 7.0, device=DEV, dtype=torch.float64)
        K.counter_add_snapshot(ctr, snap, v=2, zero=z[:nz])
        assert ctr.item() == 43 and snap.item() == 43
        assert torch.all(z[:nz] == 0) and torch.all(z[nz:] == 7.0)


def test_grad_norm_clip_full_grid_repeated(K):
    """aw_grad_norm_clip over the full grid of AW_NORM_WS partials and two segments, called repeatedly (as graph
    replays do): the f64 norm and the clip coefficient every time."""
    n = 1024 * 512 * 4 * 3 + 8
    g = torch.tensor(gen.normal(77, (n,), 1.0), device=DEV)
    off = torch.tensor([0, n // 2], device=DEV, dtype=torch.int64)
    ln = torch.tensor([n // 2 - 4, n - n // 2], device=DEV, dtype=torch.int64)
    act = torch.tensor([1, 1], device=DEV, dtype=torch.int32)
    g[n // 2 - 4:n // 2] = 0.0                      # the padding after segment 0 is zero, as the header requires
    ws = torch.zeros(K.NORM_WS, device=DEV, dtype=torch.float64)
    ref = g.double().norm().item()
    for max_norm in (1.0, 1e9, 0.5):
        norm, coef = torch.empty((), device=DEV), torch.empty((), device=DEV)
        K.grad_norm_clip(g, off, ln, act, 2, max_norm, ws, norm, coef)
        np.testing.assert_allclose(norm.item(), ref, rtol=1e-6)
        np.testing.assert_allclose(coef.item(), min(max_norm / (norm.item() + 1e-6), 1.0), rtol=1e-6)


@pytest.mark.parametrize("policy,G,Cout,Cin,Ntok,S,ref_layout,alpha", [
    (0, 16, 512, 512, 16 * 1024, 16, False, 1.0),     # the decoder's grouped launch at full size (auto policy)
    (1, 3, 256, 128, 1024, 8, True, 1.0),             # forced at a small shape: windows of 8, (O, I, 3) column map
    (1, 2, 512, 64, 2048, 32, False, 0.5),            # windows of 32, one channel block, alpha
    (-1, 4, 512, 512, 4096, 16, False, 1.0)])         # the generic grouped GEMM on the same form
def test_wgrad_conv3_kernel_vs_fp32_reference(policy, G, Cout, Cin, Ntok, S, ref_layout, alpha):
    """The 8-wave ping-pong decoder weight-gradient kernel (csrc/wgrad.hip, model/vq_vae_patch_embedd.py:60-74 grads)
    against a torch fp32 reference on the same bf16 operands: dW[o][j, i] += alpha sum_t dy[t][o] x[t+j-1][i] inside
    each window, the bias row sums, accumulation into a non-zero gradient, the tap-major [O][3I] layout and the
    reference's (O, I, 3) column map."""
    from arcweld import _native
    from arcweld import kernels as K
    g = torch.Generator(device=DEV).manual_seed(1234 + G)
    probs, refs = [], []
    for k in range(G):
        A = torch.randn(Ntok, Cout, device=DEV, generator=g).to(torch.bfloat16)
        x = torch.randn(Ntok, Cin, device=DEV, generator=g).to(torch.bfloat16)
        C0 = torch.randn(Cout, Cin, 3, device=DEV, generator=g)
        b0 = torch.randn(Cout, device=DEV, generator=g)
        full = A.float().t() @ _shift_taps(x.float(), S)          # [O][3I], column j*I + i
        if ref_layout:       # the reference's contiguous (O, I, 3) weight: column j*I + i -> i*3 + j
            C = C0.clone()
            kw = dict(C=C.view(Cout, 3 * Cin), col_map=(Cin, 3, 0))
            want = C0 + alpha * full.view(Cout, 3, Cin).permute(0, 2, 1)
        else:                # the optimizer's tap-major (O, 3, I) storage: contiguous rows
            C = C0.view(Cout, 3 * Cin).clone()
            kw = dict(C=C)
            want = C0.view(Cout, 3 * Cin) + alpha * full
        b = b0.clone()
        probs.append((A, x, Cout, 3 * Cin, Ntok, dict(a_trans=True, b_trans=True, conv=(Cin, S, 1, 1), accumulate=True,
                                                      a_rowsum=b, alpha=alpha, **kw)))
        refs.append((C, b, want, b0 + alpha * A.float().sum(0)))
    _native.call("aw_gemm_set_wgrad_policy", policy)
    try:
        K.gemm_grouped(probs)
        torch.cuda.synchronize()
    finally:
        _native.call("aw_gemm_set_wgrad_policy", 0)
    for C, b, want, bw in refs:
        scale = float(want.abs().max())
        torch.testing.assert_close(C, want, rtol=1e-4, atol=2e-5 * scale)
        torch.testing.assert_close(b, bw, rtol=1e-4, atol=2e-5 * float(bw.abs().max()))


@pytest.mark.parametrize("case", ["transformer_half", "transformer_full", "encoder", "ragged_small", "one_tile"])
def test_wgrad_batch_split_k_vs_fp32_reference(case):
    """aw_wgrad_batch (csrc/wgrad.hip, wgrad_tt_kernel: 256 x 256 tiles, k-aligned split-K units over persistent
    workgroups, split tiles summed by the last arriving piece) against torch fp32 on the same bf16 operands: dW[m][colmap(n)] += alpha
    sum_k dy[k][m] x[k][n] and the bias row sums, accumulated into non-zero gradients.
      transformer_half: the four Linear kinds of 4 blocks at d 512 (model/transformer_block.py:28-30,76-77 grads),
                        K = 51 x 321 tokens (ragged: not a multiple of the 32-token stage), 192 tiles x 4 splits;
      transformer_full: all 8 blocks in one launch (32 problems, the single-GPU step's batch): 384 tiles x 2 splits;
      encoder:          the 16 centre-tap convs (model/vq_vae_patch_embedd.py:65,68), K 16384, half of them through
                        the reference's (O, I, 3) column map (the scalar epilogue), alpha 0.5;
      ragged_small:     K = 37 (two stages, the second mostly past K), mixed shapes, no split;
      one_tile:         a single tile over K = 8200 (four pieces meet in one fix-up)."""
    from arcweld import kernels as K
    g = torch.Generator(device=DEV).manual_seed(4321)
    d = 512
    if case in ("transformer_half", "transformer_full"):
        Kt, alpha = 51 * 321, 1.0
        shapes = [(3 * d, d), (d, d), (4 * d, d), (d, 4 * d)] * (4 if case == "transformer_half" else 8)
    elif case == "encoder":
        Kt, alpha = 16384, 0.5
        shapes = [(d, d)] * 16
    elif case == "ragged_small":
        Kt, alpha = 37, 1.0
        shapes = [(256, 768), (512, 256), (256, 256)]
    else:
        Kt, alpha = 8200, 1.0
        shapes = [(256, 256)]
    probs, refs = [], []
    for i, (M, N) in enumerate(shapes):
        A = torch.randn(Kt, M, device=DEV, generator=g).to(torch.bfloat16)
        x = torch.randn(Kt, N, device=DEV, generator=g).to(torch.bfloat16)
        b0 = torch.randn(M, device=DEV, generator=g)
        full = A.float().t() @ x.float()
        if case == "encoder" and i % 2:      # contiguous (O, I, 3) conv weight: column n lands at n*3 + 1
            C0 = torch.randn(M, N, 3, device=DEV, generator=g)
            C = C0.clone()
            kw = dict(C=C.view(M, 3 * N), col_map=(0, 3, 1))
            want = C0.clone()
            want[:, :, 1] += alpha * full
        else:
            C0 = torch.randn(M, N, device=DEV, generator=g)
            C = C0.clone()
            kw = dict(C=C)
            want = C0 + alpha * full
        b = b0.clone()
        probs.append((A, x, M, N, Kt, dict(a_trans=True, b_trans=True, accumulate=True, a_rowsum=b, alpha=alpha,
                                           **kw)))
        refs.append((C, b, C0, want, b0, b0 + alpha * A.float().sum(0)))
    K.wgrad_batch(probs)
    torch.cuda.synchronize()
    for C, b, C0, want, b0, bw in refs:
        scale = float(want.abs().max())
        torch.testing.assert_close(C, want, rtol=1e-4, atol=2e-5 * scale)
        torch.testing.assert_close(b, bw, rtol=1e-4, atol=2e-5 * float(bw.abs().max()))
    # a second launch reuses the self-resetting per-tile arrival counters: the same sums are added again
    K.wgrad_batch(probs)
    torch.cuda.synchronize()
    for C, b, C0, want, b0, bw in refs:
        want2, bw2 = 2 * want - C0, 2 * bw - b0
        torch.testing.assert_close(C, want2, rtol=1e-4, atol=4e-5 * float(want2.abs().max()))
        torch.testing.assert_close(b, bw2, rtol=1e-4, atol=4e-5 * float(bw2.abs().max()))


def test_wgrad_batch_broken_handoff_poisons_the_tile():
    """The split-K fix-up of aw_wgrad_batch waits a bounded number of polls for its sibling pieces (csrc/wgrad.hip: the
    sc1 hand-off carries no acquire / release); a piece that runs out of them must poison its tile with NaN rather
    than sum partials that were never published.  aw_wgrad_set_spin_limit(0) forces that path on the one-tile case
    (four pieces meet in one fix-up).  In a child process: afterwards the per-tile hand-off counters of the process
    are stale, which would break the next launch of this one."""
    import os
    import subprocess
    import sys
    import textwrap
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vq-vae-transformer-arc-welding_amd")
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {pkg!r})
        import torch
        from arcweld import _native
        from arcweld import kernels as K
        g = torch.Generator(device="cuda").manual_seed(1)
        A = torch.randn(8200, 256, device="cuda", generator=g).to(torch.bfloat16)
        x = torch.randn(8200, 256, device="cuda", generator=g).to(torch.bfloat16)
        prob = lambda C: (A, x, 256, 256, 8200, dict(a_trans=True, b_trans=True, accumulate=True, C=C))
        ok = torch.zeros(256, 256, device="cuda")
        K.wgrad_batch([prob(ok)])
        bad = torch.zeros(256, 256, device="cuda")
        _native.call("aw_wgrad_set_spin_limit", 0)
        K.wgrad_batch([prob(bad)])
        torch.cuda.synchronize()
        print("RESULT", int(torch.isnan(ok).sum()), int(torch.isnan(bad).sum()))
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")]
    assert r.returncode == 0 and line, r.stdout + r.stderr
    n_ok, n_bad = (int(v) for v in line[0].split()[1:])
    assert n_ok == 0          # the default bound: a normal hand-off
    assert n_bad > 0          # the forced timeout: the tile is poisoned, loudly


@pytest.mark.parametrize("training", [True, False])
def test_unpatch_head_bf16_y_equals_f32_y(training):
    """aw_unpatch_head_*_ex with the ConvT output in bf16 (the bf16 operand mode, model/vq_vae_patch_embedd.py:24-31)
    computes exactly what the f32 passes compute on the same (bf16-representable) values: x_hat, the ConvT2 / BN
    gradients, the per-channel sums and g_y are bit-identical."""
    from arcweld import kernels as K
    B, Q, H = 64, 80, 512
    R = B * Q
    y16 = (torch.randn(R, H, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3)) * 1.3 + 0.2).to(
        torch.bfloat16)
    stats = torch.cat([torch.randn(H, device=DEV) * 0.1, torch.rand(H, device=DEV) + 0.5,
                       torch.randn(H, device=DEV) * 0.2 + 1.0, torch.randn(H, device=DEV) * 0.1])
    w2 = torch.randn(H, 5, device=DEV) * 0.05
    b2 = torch.randn(1, device=DEV)
    g = torch.randn(B, Q * 5 // 2, 2, device=DEV)
    outs = []
    for y in (y16.float(), y16):
        x_hat = torch.empty(B, Q * 5 // 2, 2, device=DEV)
        K.unpatch_head_fwd(y, Q, stats, w2, b2, x_hat)
        gsums = torch.zeros(2 * H, device=DEV, dtype=torch.float64)
        gw2, gb2 = torch.zeros(H, 5, device=DEV), torch.zeros(1, device=DEV)
        gga, gbe = torch.zeros(H, device=DEV), torch.zeros(H, device=DEV)
        K.unpatch_head_bwd1(y, Q, stats, w2, g, gsums, gw2, gb2, gga, gbe)
        gy, dby = torch.empty(R, H, device=DEV, dtype=torch.bfloat16), torch.zeros(H, device=DEV)
        K.unpatch_head_bwd2(y, Q, stats, w2, g, gsums, training, gy, dby)
        torch.cuda.synchronize()
        outs.append((x_hat, gsums, gw2, gb2, gga, gbe, gy, dby))
    # the per-channel reductions end in atomics (order varies run to run): close, not bitwise; the per-row
    # quantities (x_hat, g_y) use the same inputs in the same order
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=0, atol=0)
    for a, b in zip(outs[1][1:6], outs[0][1:6]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))
    torch.testing.assert_close(outs[1][6].float(), outs[0][6].float(), rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(outs[1][7], outs[0][7], rtol=1e-4, atol=1e-5 * float(outs[0][7].abs().max()))


@pytest.mark.parametrize("sort", [True, False])
@pytest.mark.parametrize("B,T,V,D", [(51, 321, 514, 512), (2, 7, 9, 64), (3, 40, 8194, 512), (4, 33, 30, 36),
                                     (2, 5, 7, 6), (2, 9, 40000, 64), (5, 50, 3, 256), (2, 70, 5, 1024)])
def test_embedding_forward_backward_vs_torch(B, T, V, D, sort):
    """aw_embed_fwd / aw_embed_bwd (model/embedding.py:57-59) against torch: the forward bit-exact (one f32 add per
    element; the row-vectorised kernel at D % 4 == 0, the element-wise one at D = 6), the table gradient as
    index_add_ of the row gradients.  Cases: the decoder's 51 x 321 rows into 514 table rows (~32 rows per table
    row), a tiny table with many repeats, the stress table of 8194 rows, D = 36 and D = 6, a 40000-row table (past the
    sorted form's LDS bins: its atomic fallback).  Both table-gradient forms: the counting sort (aw_embed_bwd_sorted;
    D = 6 / 36 / 64 take its fallback) and the atomic one.  Ids leave one table row unused, which must stay unchanged."""
    from arcweld import kernels as K
    g = torch.Generator(device="cuda").manual_seed(V + D)
    ids = torch.randint(0, V - 1, (B, T), device="cuda", generator=g)       # row V-1 is never used
    W = torch.randn(V, D, device="cuda", generator=g)
    pe = torch.randn(T, D, device="cuda", generator=g)
    x = torch.empty(B * T, D, device="cuda")
    K.embed_fwd(ids, W, pe, x)
    ref = (W[ids] + pe[None]).reshape(B * T, D)
    assert torch.equal(x, ref)
    dx = torch.randn(B * T, D, device="cuda", generator=g)
    prior = torch.randn(V, D, device="cuda", generator=g)
    dw = prior.clone()
    K.embed_bwd(ids, dx, dw, sort=sort)
    want = prior.clone().index_add_(0, ids.reshape(-1), dx)
    torch.testing.assert_close(dw, want, rtol=1e-5, atol=1e-4)
    assert torch.equal(dw[V - 1], prior[V - 1])


@pytest.mark.parametrize("B,T,V,D,dt", [(51, 321, 514, 512, torch.bfloat16), (3, 17, 30, 256, torch.float32),
                                        (2, 9, 11, 768, torch.bfloat16), (2, 5, 7, 1024, torch.float32)])
def test_embed_ln_fused_matches_the_two_launches(B, T, V, D, dt):
    """aw_embed_ln_fwd (the decoder's embedding with block 0's ln_1 fused) against aw_embed_fwd followed by
    aw_layernorm_fwd on the same inputs: x, y, mean and rstd bit-identical (the same per-element add and the vector
    LayerNorm's order of operations), at every d_model the fused form accepts and both operand dtypes."""
    from arcweld import kernels as K
    g = torch.Generator(device="cuda").manual_seed(B * T + D)
    ids = torch.randint(0, V, (B, T), device="cuda", generator=g)
    W = torch.randn(V, D, device="cuda", generator=g)
    pe = torch.randn(T + 3, D, device="cuda", generator=g)          # a longer table: rows t < T are read
    w = 1 + 0.1 * torch.randn(D, device="cuda", generator=g)
    b = 0.1 * torch.randn(D, device="cuda", generator=g)
    R = B * T
    x0, y0, m0, r0 = torch.empty(R, D, device="cuda"), torch.empty(R, D, device="cuda", dtype=dt), \
        torch.empty(R, device="cuda"), torch.empty(R, device="cuda")
    K.embed_fwd(ids, W, pe, x0)
    K.layernorm_fwd(x0, w, b, 1e-5, y0, m0, r0)
    x1, y1, m1, r1 = (torch.full_like(t, float("nan")) for t in (x0, y0, m0, r0))
    K.embed_ln_fwd(ids, W, pe, x1, w, b, 1e-5, y1, m1, r1)
    for got, want in ((x1, x0), (y1, y0), (m1, m0), (r1, r0)):
        assert torch.equal(got, want)


@pytest.mark.parametrize("R,V,D", [(16371, 514, 512), (300, 3, 256), (4000, 8194, 1024), (7, 15360, 768)])
def test_embed_sort_segsum_halves(R, V, D):
    """aw_embed_sort + aw_embed_bwd_segsum (the two halves of aw_embed_bwd_sorted, callable apart) against index_add_: the offsets are the exclusive prefix sums of the id counts, every row index
    lands in its id's segment exactly once, and the table gradient matches; cases: the decoder's 16371 x 514, a
    3-row table with ~100-row segments (several 64-entry batches per segment), the 8194-row stress table at D 1024,
    the largest table the LDS bins take."""
    from arcweld import kernels as K
    g = torch.Generator(device="cuda").manual_seed(R + V)
    ids = torch.randint(0, V, (R,), device="cuda", generator=g)
    work = torch.full((V + 1 + R,), -7, device="cuda", dtype=torch.int32)
    K.embed_sort(ids, V, work)
    cnt = torch.bincount(ids, minlength=V)
    off = torch.zeros(V + 1, dtype=torch.int64, device="cuda")
    off[1:] = torch.cumsum(cnt, 0)
    assert torch.equal(work[:V + 1].long(), off)
    ord_ = work[V + 1:].long()
    assert torch.equal(torch.sort(ord_).values, torch.arange(R, device="cuda"))
    seg = torch.repeat_interleave(torch.arange(V, device="cuda"), cnt)
    assert torch.equal(ids[ord_], seg)
    dx = torch.randn(R, D, device="cuda", generator=g)
    prior = torch.randn(V, D, device="cuda", generator=g)
    dw = prior.clone()
    K.embed_bwd_segsum(work, dx, dw)
    torch.testing.assert_close(dw, prior.clone().index_add_(0, ids, dx), rtol=1e-5, atol=1e-4)
