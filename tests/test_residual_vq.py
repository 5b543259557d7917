"""ResidualVQLightning / --use-improved-vq (reference model/vector_quantizer.py:9-56, vq_vae_patch_embedd.py:132-136).

PARITY UNPINNED against the reference: it wraps vector-quantize-pytorch's ResidualVQ, which is not installed here and
for which the reference holds no test or fixture.  The HIP path (arcweld/residual_vq.py, csrc/rvq.hip) is checked
against the CPU restatement of the library's published algorithm in oracle/residual_vq.py: k-means init, nearest-code
assignment, EMA codebook update with Laplace smoothing, dead-code replacement (same counter-hash rows), commitment
loss, straight-through backward, and the whole VQ-VAE train step with the residual VQ plugged into oracle/vqvae.py.
Inputs are built so that nearest codes are unambiguous (well-separated clusters), so indices compare exactly."""
import numpy as np
import pytest
import torch

from oracle import gen
from oracle import residual_vq as orv
from oracle import vqvae as ov

KW = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)


# ------------------------------------------------------------------------------------------------ CPU
def test_improved_vq_module_layout():
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, batch_norm=False, use_improved_vq=True, kmeans_iters=10,
                   threshold_ema_dead_code=2, **KW)
    sd = m.state_dict()
    pre = "vector_quantization.vq.layers.0._codebook."
    assert tuple(sd[pre + "embed"].shape) == (1, 64, 16)
    assert tuple(sd[pre + "embed_avg"].shape) == (1, 64, 16)
    assert tuple(sd[pre + "cluster_size"].shape) == (1, 64)
    assert float(sd[pre + "initted"]) == 0.0                     # k-means init pending
    assert "vector_quantization.embedding.weight" not in sd
    # no codebook parameter: the split of the overlapped all-reduce starts at the decoder's 1x1 conv
    assert m.backward_split_parameter() is m.decoder[0].weight
    vq = m.vector_quantization
    assert (vq.n_e, vq.e_dim, vq.kmeans_init, vq.kmeans_iters, vq.threshold_ema_dead_code, vq.num_quantizers) == \
        (64, 16, True, 10, 2, 1)
    # every non-VQ key matches the plain model's
    plain = VQVAEPatch(input_dim=2, learning_rate=1e-3, batch_norm=False, **KW).state_dict()
    assert {k for k in plain if not k.startswith("vector_quantization")} == \
        {k for k in sd if not k.startswith("vector_quantization")}


def test_oracle_kmeans_recovers_separated_clusters():
    rng = np.random.default_rng(0)
    C = rng.normal(size=(8, 4)).astype(np.float32) * 5
    lab = np.repeat(np.arange(8), 50)
    x = (C[lab] + 0.01 * rng.normal(size=(400, 4))).astype(np.float32)
    means, bins = orv.kmeans(x, 8, 3, init_rows=np.arange(8) * 50 + 7)
    np.testing.assert_allclose(means, C, atol=0.01)
    assert bins.tolist() == [50.0] * 8
    with pytest.raises(ValueError):
        orv.kmeans(x, 8, 0, init_rows=np.arange(8))


def test_oracle_dead_code_rows_are_distinct_and_stratified():
    expired = np.zeros(100, bool)
    expired[[3, 10, 11, 50, 99]] = True
    rows = orv.dead_code_rows(expired, 1000, salt=5, ctr=7)
    picked = rows[expired]
    assert (rows[~expired] == -1).all()
    assert len(set(picked.tolist())) == 5
    for j, r in enumerate(picked):
        assert j * 200 <= r < (j + 1) * 200
    assert not np.array_equal(picked, orv.dead_code_rows(expired, 1000, salt=5, ctr=8)[expired])


# ------------------------------------------------------------------------------------------------ GPU
def _clustered(nq, seed=0):
    """Hierarchical, balanced clusters: layer 1 sees 64 clusters (c1); with nq = 2 every point also carries one of
    64 sub-cluster offsets (c2), each (l1, l2) pair exactly once, so the residual left by layer 1 is c2[l2] minus
    the same mean in every l1 cluster: layer 2 sees 64 clean clusters too."""
    rng = np.random.default_rng(seed)
    D = 32
    c1 = rng.normal(size=(64, D)).astype(np.float32) * 3
    c2 = rng.normal(size=(64, D)).astype(np.float32) * 0.3
    l1 = np.repeat(np.arange(64), 64)
    l2 = np.tile(np.arange(64), 64)
    z = c1[l1] + (c2[l2] if nq > 1 else 0) + 1e-3 * rng.normal(size=(4096, D))
    perm = rng.permutation(4096)
    z, l1, l2 = z[perm].astype(np.float32), l1[perm], l2[perm]
    init1 = np.array([np.flatnonzero(l1 == c)[0] for c in range(64)])
    init2 = np.array([np.flatnonzero(l2 == c)[0] for c in range(64)])
    return z, l1, l2, init1, init2


@pytest.mark.gpu
@pytest.mark.parametrize("nq", [1, 2])
def test_residual_vq_training_steps_match_oracle(nq):
    from arcweld.residual_vq import ResidualVQ
    z, l1, l2, init1, init2 = _clustered(nq)
    rvq = ResidualVQ(nq, 32, 64, kmeans_init=True, kmeans_iters=3, threshold_ema_dead_code=2).cuda().train()
    inits = [init1, init2][:nq]
    for layer, rows in zip(rvq.layers, inits):
        layer._codebook.init_rows = torch.tensor(rows)
    books = [orv.Codebook(64, 32, 3, 2) for _ in range(nq)]
    salts = [0x5EED + 7919 * i for i in range(nq)]
    zt = torch.tensor(z, device="cuda")
    for step in range(3):
        out, idx, losses, _ = rvq.quantize_rows(zt, True)
        o_out, o_idx, o_losses, _, _ = orv.residual_vq_forward(books, z, True, init_rows=inits, salts=salts,
                                                               ctr=step + 1)
        assert np.array_equal(idx.cpu().numpy(), o_idx), step
        np.testing.assert_allclose(out.cpu().numpy(), o_out, atol=1e-5)
        np.testing.assert_allclose(losses.cpu().numpy(), o_losses, rtol=1e-4, atol=1e-9)
        for layer, cb in zip(rvq.layers, books):
            c = layer._codebook
            np.testing.assert_allclose(c.cluster_size[0].cpu().numpy(), cb.cluster_size, rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(c.embed_avg[0].cpu().numpy(), cb.embed_avg, rtol=1e-4, atol=1e-4)
            np.testing.assert_allclose(c.embed[0].cpu().numpy(), cb.embed, rtol=1e-4, atol=1e-5)
            assert float(c.initted) == 1.0


@pytest.mark.gpu
def test_dead_codes_take_the_oracle_rows():
    """Codes whose cluster vanishes from the batch decay below the threshold and are replaced by the same batch
    rows (counter-hash strata) in both paths."""
    from arcweld.residual_vq import ResidualVQ
    z, l1, _, init1, _ = _clustered(1, seed=3)
    rvq = ResidualVQ(1, 32, 64, kmeans_init=True, kmeans_iters=2, threshold_ema_dead_code=60).cuda().train()
    rvq.layers[0]._codebook.init_rows = torch.tensor(init1)
    book = orv.Codebook(64, 32, 2, 60)
    keep = l1 < 32                      # the second batch draws only from clusters 0..31
    z2 = np.concatenate([z[keep], z[keep]])
    for step, batch in enumerate((z, z2)):
        rvq.quantize_rows(torch.tensor(batch, device="cuda"), True)
        orv.residual_vq_forward([book], batch, True, init_rows=[init1], salts=[0x5EED], ctr=step + 1)
    c = rvq.layers[0]._codebook
    emb = c.embed[0].cpu().numpy()
    cs = c.cluster_size[0].cpu().numpy()
    assert (book.cluster_size[32:] == 60).all() and (cs[32:] == 60).all()       # expired and reset
    np.testing.assert_array_equal(emb[32:], book.embed[32:])                     # the same replacement rows
    rows = {tuple(r) for r in z2}
    assert all(tuple(r) in rows for r in emb[32:])
    np.testing.assert_allclose(emb[:32], book.embed[:32], rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_residual_vq_backward_matches_oracle():
    from arcweld import kernels as K
    rng = np.random.default_rng(1)
    nq, N, D = 3, 1000, 16
    res = rng.normal(size=(nq, N, D)).astype(np.float32)
    q = rng.normal(size=(nq, N, D)).astype(np.float32)
    g = rng.normal(size=(N, D)).astype(np.float32)
    gl = np.array([0.5, -2.0, 3.0], np.float32)
    dz = torch.empty(N, D, device="cuda")
    K.rvq_backward(*(torch.tensor(a, device="cuda") for a in (res, q, g, gl)), dz)
    np.testing.assert_allclose(dz.cpu().numpy(), orv.residual_vq_backward(res, q, g, gl), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_standalone_module_forward_backward():
    """ResidualVQLightning as a module (autograd path): reference output tuple, straight-through gradient."""
    from model.vector_quantizer import ResidualVQLightning
    z, _, _, init1, _ = _clustered(1, seed=5)
    m = ResidualVQLightning(n_e=64, e_dim=32, kmeans_init=True, kmeans_iters=2, threshold_ema_dead_code=2).cuda()
    m.vq.layers[0]._codebook.init_rows = torch.tensor(init1)
    x = torch.tensor(z, device="cuda").view(64, 64, 32).requires_grad_(True)
    loss, zq, perp, enc, idx = m(x)
    assert perp is None and enc is None
    assert tuple(loss.shape) == (1, 1) and tuple(idx.shape) == (64, 64, 1) and zq.shape == x.shape
    g = torch.randn_like(zq)
    (zq * g).sum().add(loss.sum() * 2.0).backward()
    ref = orv.residual_vq_backward(x.detach().reshape(1, -1, 32).cpu().numpy(),
                                   zq.detach().reshape(1, -1, 32).cpu().numpy(), g.reshape(-1, 32).cpu().numpy(),
                                   np.array([2.0], np.float32))
    np.testing.assert_allclose(x.grad.reshape(-1, 32).cpu().numpy(), ref, rtol=1e-5, atol=1e-7)
    ood, zq2, idx2, closs = m.eval().forward_ood(x.detach())
    assert tuple(ood.shape) == (64,) and float(closs.sum()) == 0.0


def _improved_model(wseed, iters=3):
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, use_improved_vq=True,
                   kmeans_iters=iters, threshold_ema_dead_code=2, **KW)
    sd = ov.det_state_dict(ov.VQVAEConfig(**KW), wseed)
    missing, unexpected = m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()
                                             if not k.startswith("vector_quantization")}, strict=False)
    assert all(k.startswith("vector_quantization.vq.") for k in missing) and not unexpected
    return m.cuda().train(), sd


@pytest.mark.gpu
def test_vqvae_train_step_with_residual_vq_matches_oracle():
    """The fused VQ-VAE step with --use-improved-vq: x_hat, loss (mse + commitment) and every parameter gradient
    against oracle/vqvae.py with the residual VQ plugged in (codebook state of before the step), then the EMA
    codebook update against oracle/residual_vq.py on the oracle's own z_e."""
    from arcweld.precision import operands
    m, sd = _improved_model(401)
    x = torch.tensor(gen.windows(402, 8), device="cuda")
    cfg = ov.VQVAEConfig(**KW)
    # codebook state before the step: 64 encoder outputs of another batch (initted, no k-means on this batch)
    z_prev = ov.vqvae_train_step_grads(sd, gen.windows(403, 8), cfg)[0]["z_e"].reshape(-1, 16)[::2][:64]
    cb = m.vector_quantization.vq.layers[0]._codebook
    with torch.no_grad():
        cb.embed[0].copy_(torch.tensor(z_prev))
        cb.embed_avg[0].copy_(torch.tensor(z_prev) * 5.0)
        cb.cluster_size.fill_(5.0)
        cb.initted.fill_(1.0)
    cb._initted_host = None
    with operands(torch.float32):
        emb, x_hat, perp = m(x)
        assert perp is None
        loss = torch.nn.functional.mse_loss(x_hat, x) + emb
        loss.backward()
    out, grads, _ = ov.vqvae_train_step_grads(sd, x.cpu().numpy(), cfg, quantizer=orv.torch_quantizer([z_prev]))
    np.testing.assert_allclose(x_hat.detach().cpu().numpy(), out["x_hat"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(loss.detach()), float(out["loss"]), rtol=1e-4)
    assert np.array_equal(m._last_indices.cpu().numpy(), out["idx"].reshape(-1))
    for name, p in m.named_parameters():
        ref = grads[name]
        rel = np.linalg.norm(p.grad.cpu().numpy() - ref) / (np.linalg.norm(ref) + 1e-20)
        assert rel < 2e-3 or np.abs(ref).max() < 1e-6, (name, rel)
    book = orv.Codebook(64, 16, 3, 2)
    book.embed, book.embed_avg = z_prev.astype(np.float32), (z_prev * 5.0).astype(np.float32)
    book.cluster_size, book.initted = np.full(64, 5.0, np.float32), True
    book.forward(out["z_e"].reshape(-1, 16), True, salt=0x5EED, ctr=1)
    np.testing.assert_allclose(cb.cluster_size[0].cpu().numpy(), book.cluster_size, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(cb.embed[0].cpu().numpy(), book.embed, rtol=1e-3, atol=1e-4)


@pytest.mark.gpu
def test_improved_vq_trains_graphed_and_tokenizes():
    """k-means init on the first (eager) step, then captured steps replay the EMA update; eager and graphed runs
    follow the same trajectory; tokenization uses the residual VQ's codebook."""
    from arcweld.trainer import Trainer
    xs = [torch.tensor(gen.windows(900 + i, 16), device="cuda") for i in range(5)]
    runs = []
    for graphed in (False, True):
        torch.manual_seed(11)
        m, _ = _improved_model(411)
        m.vector_quantization.vq.layers[0]._codebook.init_rows = torch.arange(64) * 3
        tr = Trainer(gradient_clip_val=0.7)
        tr.setup_optimizer(m)
        losses = []
        for x in xs:
            if graphed:
                losses.append(float(tr.graphed_step(m, x, 1.0)))
            else:
                losses.append(float(tr.micro_step(m, x, 0, 1.0)))
                tr.optimizer_step(m)
        runs.append((losses, {k: v.detach().clone() for k, v in m.state_dict().items()}, m))
    (l0, s0, _), (l1, s1, m1) = runs
    assert all(np.isfinite(l0))
    np.testing.assert_allclose(l1, l0, rtol=1e-4)
    for k in s0:
        torch.testing.assert_close(s1[k].float(), s0[k].float(), rtol=1e-4, atol=1e-5, msg=k)
    ids = m1.eval().encode_ids(xs[0])
    assert ids.shape == (16, 16) and int(ids.max()) < 64


def _rvq_dp_worker(rank, world, port, z, init_rows, out):
    import os
    import torch.distributed as dist
    from arcweld.residual_vq import ResidualVQ
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rvq = ResidualVQ(1, 32, 64, kmeans_init=True, kmeans_iters=3, threshold_ema_dead_code=2).cuda().train()
        rvq.layers[0]._codebook.init_rows = torch.tensor(init_rows)      # rank 0's rows seed the broadcast means
        n = z.shape[0] // world
        half = torch.tensor(z[rank * n:(rank + 1) * n], device="cuda")
        for _ in range(3):
            rvq.quantize_rows(half, True)
        torch.cuda.synchronize()
        c = rvq.layers[0]._codebook
        out[rank] = {k: getattr(c, k).cpu().clone() for k in ("embed", "embed_avg", "cluster_size")}
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_residual_vq_data_parallel_world2_matches_full_batch():
    """Data parallel (two ranks over gloo sharing cuda:0): k-means and the EMA all-reduce bins and per-code sums, so
    both ranks hold the codebook a single process gets from the whole batch."""
    import socket
    import torch.multiprocessing as mp
    from arcweld.residual_vq import ResidualVQ
    z, l1, _, _, _ = _clustered(1, seed=7)
    init = np.array([np.flatnonzero(l1[:2048] == c)[0] for c in range(64)])     # rows of rank 0's half
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.Manager().dict()
    mp.spawn(_rvq_dp_worker, args=(2, port, z, init, out), nprocs=2, join=True)
    ref = ResidualVQ(1, 32, 64, kmeans_init=True, kmeans_iters=3, threshold_ema_dead_code=2).cuda().train()
    ref.layers[0]._codebook.init_rows = torch.tensor(init)
    full = torch.tensor(z, device="cuda")
    for _ in range(3):
        ref.quantize_rows(full, True)
    c = ref.layers[0]._codebook
    for k in ("embed", "embed_avg", "cluster_size"):
        torch.testing.assert_close(out[0][k], out[1][k], rtol=0, atol=0, msg=k)
        torch.testing.assert_close(out[0][k], getattr(c, k).cpu(), rtol=1e-5, atol=1e-5, msg=k)
