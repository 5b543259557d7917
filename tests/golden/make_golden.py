"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE model modules.

Run ONLY in the build container (it needs /root/reference, which never travels to the GPU box):

    python tests/golden/make_golden.py

The reference modules subclass ``lightning.pytorch.LightningModule`` and import ``torchmetrics`` and
``vector_quantize_pytorch``, none of which is installed.  A throw-away stub package for those three names is
written to a temporary directory and put on ``sys.path`` ahead of /root/reference.
The stubs carry no arithmetic: ``LightningModule`` is ``nn.Module`` plus no-op ``save_hyperparameters``/``log``
and a ``device`` property; ``ResidualVQ`` raises (the improved-VQ branch is out of scope).

Inputs come from ``oracle/gen.py`` (seed + parameter name), so only outputs are stored.  Every fixture is
computed in fp32 on CPU with torch's deterministic CPU kernels.
"""
from __future__ import annotations

import os
import sys
import tempfile
import textwrap

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle import gen  # noqa: E402

_SHIM = {
    "lightning/__init__.py": "from lightning import pytorch\n",
    "lightning/pytorch/__init__.py": textwrap.dedent(
        """
        import torch
        from torch import nn
        class LightningModule(nn.Module):
            def save_hyperparameters(self, *a, **k):
                pass
            def log(self, *a, **k):
                pass
            @property
            def device(self):
                for p in self.parameters():
                    return p.device
                return torch.device('cpu')
        class LightningDataModule:
            pass
        """),
    "torchmetrics/__init__.py": "",
    "torchmetrics/functional/__init__.py": textwrap.dedent(
        """
        def accuracy(*a, **k):
            raise RuntimeError('metrics stub: logging only')
        def f1_score(*a, **k):
            raise RuntimeError('metrics stub: logging only')
        """),
    "vector_quantize_pytorch/__init__.py": textwrap.dedent(
        """
        class ResidualVQ:
            def __init__(self, *a, **k):
                raise RuntimeError('improved VQ is out of scope (vector-quantize-pytorch not installed)')
        """),
    # dataloader/utils.py reads the data path from a .env file; every call here passes data_directory_path
    "dotenv/__init__.py": "def dotenv_values(*a, **k):\n    return {}\n",
}


def install_shim() -> str:
    d = tempfile.mkdtemp(prefix="ref_shim_")
    for rel, src in _SHIM.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(src)
    sys.path.insert(0, REF)
    sys.path.insert(0, d)
    return d


def load_det_state(model: torch.nn.Module, base: int) -> None:
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        if k.endswith(".attn.bias") or k.endswith("positional_embedding.pe"):
            new[k] = v                      # constant buffers (causal mask, sinusoid table) keep their values
        else:
            new[k] = torch.from_numpy(gen.param_value(base, k, tuple(v.shape))).to(v.dtype)
    model.load_state_dict(new)


def grads_of(model: torch.nn.Module, prefix: str = "grad/") -> dict:
    out = {}
    for n, p in model.named_parameters():
        if p.grad is not None:
            out[prefix + n] = p.grad.detach().numpy().copy()
    return out


def top2_gap(z: np.ndarray, E: np.ndarray) -> np.ndarray:
    zt = torch.from_numpy(z)
    Et = torch.from_numpy(E)
    d = torch.sum(zt ** 2, dim=1, keepdim=True) + torch.sum(Et ** 2, dim=1) - 2 * torch.matmul(zt, Et.t())
    v, _ = torch.topk(d, 2, dim=1, largest=False)
    return (v[:, 1] - v[:, 0]).numpy().astype(np.float32)


def save(name: str, **arrays) -> None:
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


# --------------------------------------------------------------------------------------------------
def case_vq_small(VectorQuantizer):
    torch.manual_seed(0)
    B, S, D, K, beta = 16, 16, 16, 64, 0.25
    vq = VectorQuantizer(n_e=K, e_dim=D, beta=beta)
    E = gen.uniform(101, (K, D), -0.5, 0.5)
    vq.embedding.weight.data.copy_(torch.from_numpy(E))
    z = torch.from_numpy(gen.normal(102, (B, S, D), 0.5)).requires_grad_(True)
    g_zq = torch.from_numpy(gen.normal(103, (B, S, D), 1.0))
    g_loss = 1.3
    loss, zq, perp, onehot, idx = vq(z)
    obj = g_loss * loss + (zq * g_zq).sum()
    obj.backward()
    save("vq_small.npz", idx=idx.numpy().astype(np.int64), z_q=zq.detach().numpy(), loss=loss.detach().numpy(),
         perplexity=perp.detach().numpy(), onehot_rowsum=onehot.sum(1).numpy(), dz=z.grad.numpy(),
         dE=vq.embedding.weight.grad.numpy(), g_loss=np.float32(g_loss))


def case_vq_idx(VectorQuantizer):
    out = {}
    # Encoder-like z (std ~0.08) against (a) the reference init codebook U(+-1/K) and (b) a trained-like one.
    for tag, K, D, N, eseed, estd in (("K512_D64_init", 512, 64, 16384, 201, None),
                                      ("K512_D64_trained", 512, 64, 16384, 202, 0.08),
                                      ("K8192_D256_trained", 8192, 256, 4096, 203, 0.05)):
        z = gen.normal(210 + K, (N, D), 0.08)
        if estd is None:
            E = gen.uniform(eseed, (K, D), -1.0 / K, 1.0 / K)
        else:
            E = gen.normal(eseed, (K, D), estd)
        vq = VectorQuantizer(n_e=K, e_dim=D, beta=0.25)
        vq.embedding.weight.data.copy_(torch.from_numpy(E))
        with torch.no_grad():
            loss, zq, perp, _, idx = vq(torch.from_numpy(z).view(N // 16, 16, D))
        out[f"idx_{tag}"] = idx.view(-1).numpy().astype(np.int16)
        out[f"gap_{tag}"] = top2_gap(z, E)
        out[f"loss_{tag}"] = loss.numpy()
        out[f"perplexity_{tag}"] = perp.numpy()
    save("vq_idx.npz", **out)


def vqvae_kwargs(H, K, D, R, P, bn, dropout=0.0):
    return dict(hidden_dim=H, input_dim=2, num_embeddings=K, embedding_dim=D, n_resblocks=R,
                learning_rate=1e-3, dropout_p=dropout, patch_size=P, seq_len=200, batch_norm=bn, beta=0.25)


def run_vqvae(VQVAEPatch, cfg, B, wseed, xseed, store_full_grads=True):
    torch.manual_seed(0)
    m = VQVAEPatch(**cfg)
    load_det_state(m, wseed)
    m.train()
    x = torch.from_numpy(gen.windows(xseed, B))
    captured = {}

    def hook(mod, inp, out):
        captured["idx"] = out[4].detach().view(-1).numpy().copy()
        captured["z_e"] = inp[0].detach().numpy().copy()

    h = m.vector_quantization.register_forward_hook(hook)
    emb_loss, x_hat, perp = m(x)
    h.remove()
    recon = torch.nn.functional.mse_loss(x_hat, x)
    loss = recon + emb_loss
    loss.backward()
    out = dict(x_hat=x_hat.detach().numpy(), emb_loss=emb_loss.detach().numpy(), perplexity=perp.detach().numpy(),
               recon=recon.detach().numpy(), loss=loss.detach().numpy(), idx=captured["idx"].astype(np.int64),
               z_e=captured["z_e"])
    grads = grads_of(m)
    if store_full_grads:
        out.update(grads)
    else:
        for k, g in grads.items():
            out[k.replace("grad/", "gnorm/")] = np.float64(np.linalg.norm(g.astype(np.float64)))
            out[k.replace("grad/", "gslice/")] = g.reshape(-1)[:64].copy()
    for k, v in m.state_dict().items():
        if "running" in k or "num_batches" in k:
            out["state/" + k] = v.numpy()
    m.eval()
    with torch.no_grad():
        e2, xh2, p2 = m(x)
    out["eval_x_hat"] = xh2.numpy()
    out["eval_emb_loss"] = e2.numpy()
    return out


def case_vqvae(VQVAEPatch):
    save("vqvae_small.npz", **run_vqvae(VQVAEPatch, vqvae_kwargs(64, 64, 16, 2, 25, False), 8, 301, 302))
    save("vqvae_small_bn.npz", **run_vqvae(VQVAEPatch, vqvae_kwargs(64, 64, 16, 2, 25, True), 8, 303, 304))
    save("vqvae_small_p10.npz", **run_vqvae(VQVAEPatch, vqvae_kwargs(64, 64, 16, 1, 10, False), 4, 305, 306))
    save("vqvae_small_p50.npz", **run_vqvae(VQVAEPatch, vqvae_kwargs(64, 64, 16, 1, 50, False), 4, 307, 308))
    save("vqvae_full_b4.npz", **run_vqvae(VQVAEPatch, vqvae_kwargs(512, 512, 64, 8, 25, False), 4, 309, 310,
                                          store_full_grads=False))


def run_decoder(MyTransformerDecoder, cfg, B, wseed, xseed, store_full_grads=True):
    out = {}
    torch.manual_seed(0)
    m = MyTransformerDecoder(**cfg)
    load_det_state(m, wseed)
    m.train()
    T, V = cfg["seq_len"], cfg["n_classes"]
    x = torch.from_numpy(gen.randint(xseed, (B, T), 0, V))
    y = torch.from_numpy(gen.randint(xseed + 1, (B, T), 0, V))
    y[:, -3:] = -1                                       # exercise ignore_index=-1
    cond = torch.from_numpy(gen.randint(xseed + 2, (B,), 0, 2))
    for task in ("generate", "classification"):
        m.zero_grad(set_to_none=True)
        if task == "generate":
            m.switch_to_generate()
            loss, logits, _ = m.step_task_gen((x, cond, y))
        else:
            m.switch_to_classification()
            loss, logits, _ = m.step_task_class((x, cond, y))
        loss.backward()
        t = "gen" if task == "generate" else "cls"
        out[f"{t}/loss"] = loss.detach().numpy()
        if store_full_grads or t == "cls":
            out[f"{t}/logits"] = logits.detach().numpy()
        else:
            out[f"{t}/logits_slice"] = logits.detach()[:, :, :32].numpy().copy()
            out[f"{t}/logits_lastrow"] = logits.detach()[:, -1, :].numpy().copy()
        grads = grads_of(m, prefix=f"{t}/grad/")
        if store_full_grads:
            out.update(grads)
        else:
            for k, g in grads.items():
                out[k.replace("/grad/", "/gnorm/")] = np.float64(np.linalg.norm(g.astype(np.float64)))
                out[k.replace("/grad/", "/gslice/")] = g.reshape(-1)[:64].copy()
        out[f"{t}/grad_names"] = np.array(sorted(k.split("/grad/")[1] for k in grads))
    return out


def case_decoder(MyTransformerDecoder):
    save("decoder_small.npz", **run_decoder(MyTransformerDecoder, dict(
        d_model=64, n_classes=34, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0, att_dropout=0.0), 4, 401, 402))
    save("decoder_small_bias.npz", **run_decoder(MyTransformerDecoder, dict(
        d_model=64, n_classes=34, seq_len=33, n_blocks=2, n_head=4, res_dropout=0.0, att_dropout=0.0,
        class_h_bias=True), 3, 403, 404))
    save("decoder_full_b2.npz", **run_decoder(MyTransformerDecoder, dict(
        d_model=512, n_classes=514, seq_len=321, n_blocks=8, n_head=8, res_dropout=0.0, att_dropout=0.0), 2, 405, 406,
        store_full_grads=False))


def case_radam():
    """Reference optimizer semantics: torch.optim.RAdam as built by configure_optimizers (both setups) and
    Lightning's gradient_clip_val (clip_grad_norm_, L2)."""
    out = {}
    shapes = [(33, 7), (7,), (5, 3, 2)]
    for tag, betas, groups in (("vqvae", (0.9, 0.999), [(0.0, [0, 1, 2])]),
                               ("decoder", (0.9, 0.95), [(0.1, [0, 2]), (0.0, [1])])):
        params = [torch.nn.Parameter(torch.from_numpy(gen.normal(500 + i, s, 0.3))) for i, s in enumerate(shapes)]
        opt = torch.optim.RAdam([{"params": [params[i] for i in idx], "weight_decay": wd} for wd, idx in groups],
                                lr=1e-3, betas=betas)
        for step in range(8):
            for i, p in enumerate(params):
                p.grad = torch.from_numpy(gen.normal(600 + 17 * step + i, p.shape, 1.0))
            out[f"{tag}/prenorm_{step}"] = torch.nn.utils.clip_grad_norm_(params, 0.7).numpy()
            opt.step()
            for i, p in enumerate(params):
                out[f"{tag}/p{i}_step{step}"] = p.detach().numpy().copy()
    save("radam.npz", **out)


# ----------------------------------------------------------------------------- training regime
REGIME_KW = dict(d_model=32, n_classes=20, seq_len=17, n_blocks=2, n_head=4, res_dropout=0.0, att_dropout=0.0)
REGIME_STAGES = (("generate", 3), ("classification", 2))    # (task, optimizer steps); 5 micro-batches per step


def regime_batch(stage: int, step: int, micro: int):
    """Micro-batch (x, cond, y) of 4 sequences: ids in [0, 18) with start/end tokens 18/19 as
    MyLatentAutoregressiveDataset builds them (dataloader/base_dataloader.py:74-110)."""
    seed = 1000 + 100 * stage + 10 * step + micro
    ids = gen.randint(seed, (4, 16), 0, 18)
    x = np.concatenate([np.full((4, 1), 18), ids], axis=1)
    y = np.concatenate([ids, np.full((4, 1), 19)], axis=1)
    cond = gen.randint(seed + 7, (4,), 0, 2)
    return torch.from_numpy(x), torch.from_numpy(cond), torch.from_numpy(y)


def case_training_regime(MyTransformerDecoder):
    """train_transformer_mtasks.py:23-33,178-190 on the reference module: per stage a new Trainer and so a new
    optimizer (the module's own configure_optimizers: torch.optim.RAdam, betas (0.9, 0.95), wd 0.1 on Linear
    weights); Lightning automatic optimisation with accumulate_grad_batches=5 (each micro-batch loss / 5, one
    backward each), gradient_clip_val=0.8 (clip_grad_norm_ over the optimizer's parameters -- the unused head has
    grad None and is skipped), optimizer.step(), zero_grad(set_to_none=True).  Generate stage, then a
    classification stage on the same module."""
    torch.manual_seed(0)
    m = MyTransformerDecoder(**REGIME_KW)
    load_det_state(m, 1001)
    m.train()
    out = {}
    for si, (task, nsteps) in enumerate(REGIME_STAGES):
        (m.switch_to_generate if task == "generate" else m.switch_to_classification)()
        opt = m.configure_optimizers()
        params = [p for g in opt.param_groups for p in g["params"]]
        for step in range(nsteps):
            losses = []
            for micro in range(5):
                loss, _, _ = m._step(regime_batch(si, step, micro))
                (loss / 5).backward()
                losses.append(loss.item())
            out[f"s{si}/loss_{step}"] = np.array(losses, dtype=np.float32)
            out[f"s{si}/gradnorm_{step}"] = torch.nn.utils.clip_grad_norm_(params, 0.8).numpy()
            out[f"s{si}/unused_grad_is_none_{step}"] = np.array(
                (m.class_head.linear_1.weight.grad is None) if task == "generate" else (m.lm_head.weight.grad is None))
            opt.step()
            opt.zero_grad(set_to_none=True)
        for n, p in m.named_parameters():
            out[f"s{si}/param/{n}"] = p.detach().numpy().copy()
    save("training_regime.npz", **out)


# ------------------------------------------------------------------------- ASIMoW CSV format
ASIMOW_VAL = ((1, 2), (3, 1))
ASIMOW_TEST = ((2, 3),)
ASIMOW_CASES = (("reconstruction", 1), ("classification", 1), ("classification", 3))


def asimow_frame(n=90):
    """A synthetic processed_asimow_dataset.csv in the reference's column layout (experiment, welding_run, labels,
    V_0..V_199, I_0..I_199); values on a 1e-3 grid so the CSV text round-trips exactly."""
    import pandas as pd
    exp = gen.randint(1501, (n,), 1, 4)
    run = gen.randint(1502, (n,), 1, 5)
    lab = gen.randint(1503, (n,), -1, 2)
    v = np.round(gen.normal(1504, (n, 200), 3.0, 20.0).astype(np.float64), 3)
    i = np.round(gen.normal(1505, (n, 200), 30.0, 150.0).astype(np.float64), 3)
    cols = {"experiment": exp, "welding_run": run, "labels": lab}
    cols.update({f"V_{k}": v[:, k] for k in range(200)})
    cols.update({f"I_{k}": i[:, k] for k in range(200)})
    return pd.DataFrame(cols)


def case_asimow():
    """The reference's own ASIMoWDataLoader (dataloader/asimow_dataloader.py:28-206) on a synthetic CSV: CSV parse,
    (experiment, welding_run) split, per-channel StandardScaler fitted on train, cycle sequences, numpy-global-RNG
    shuffle.  Its pickle cache is written and read back by the reference inside a temporary directory (our own
    synthetic data); nothing shipped with the reference is unpickled."""
    from dataloader.asimow_dataloader import ASIMoWDataLoader, DataSplitId
    out = {}
    for task, seq in ASIMOW_CASES:
        with tempfile.TemporaryDirectory() as d:
            asimow_frame().to_csv(os.path.join(d, "processed_asimow_dataset.csv"), index=False)
            dl = ASIMoWDataLoader([DataSplitId(e, r) for e, r in ASIMOW_VAL], [DataSplitId(e, r) for e, r in ASIMOW_TEST],
                                  task=task, cycle_seq_number=seq, seed=7, data_directory_path=d)
            for name, ds in zip(("train", "val", "test"), dl.get_dataset()):
                out[f"{task}_{seq}/{name}/x"] = np.asarray(ds.data, dtype=np.float64)
                if hasattr(ds, "labels"):
                    out[f"{task}_{seq}/{name}/y"] = np.asarray(ds.labels, dtype=np.float64)
    save("asimow_split.npz", **out)


# ------------------------------------------------------------------------ Lightning checkpoint
def case_checkpoints(VQVAEPatch, MyTransformerDecoder):
    """Checkpoints in Lightning's .ckpt layout ({state_dict, hyper_parameters, epoch, global_step, ...}) built from
    the reference modules' own state_dicts and constructor arguments (what ModelCheckpoint writes and
    load_from_checkpoint reads, utils.py:30, train_transformer_mtasks.py:171), with the reference's eval outputs
    on fixed inputs.  Tensors and plain Python values only: torch.load(weights_only=True) reads them."""
    vq_kw = vqvae_kwargs(64, 64, 16, 2, 25, False, dropout=0.1)
    torch.manual_seed(0)
    m = VQVAEPatch(**vq_kw)
    load_det_state(m, 1601)
    ck = {"epoch": 3, "global_step": 120, "pytorch-lightning_version": "2.1.0",
          "state_dict": {k: v.detach().clone() for k, v in m.state_dict().items()},
          "hyper_parameters": dict(vq_kw, use_improved_vq=False, kmeans_iters=0, threshold_ema_dead_code=2),
          "loops": {}, "callbacks": {}, "optimizer_states": [], "lr_schedulers": []}
    torch.save(ck, os.path.join(HERE, "ref_vqvae_small.ckpt"))
    m.eval()
    x = torch.from_numpy(gen.windows(1602, 4))
    with torch.no_grad():
        e, xh, p = m(x)
        _, _, _, _, idx = m.vector_quantization(m.encoder(m.patch_embed(x)))
    dec_kw = dict(d_model=32, n_classes=20, seq_len=17, n_blocks=2, n_head=4, res_dropout=0.1, att_dropout=0.0,
                  learning_rate=1e-3, class_h_bias=True, class_h_dropout=False)
    torch.manual_seed(0)
    d = MyTransformerDecoder(**dec_kw)
    load_det_state(d, 1603)
    ck = {"epoch": 9, "global_step": 50, "pytorch-lightning_version": "2.1.0",
          "state_dict": {k: v.detach().clone() for k, v in d.state_dict().items()},
          "hyper_parameters": dec_kw, "loops": {}, "callbacks": {}, "optimizer_states": [], "lr_schedulers": []}
    torch.save(ck, os.path.join(HERE, "ref_decoder_small.ckpt"))
    d.eval()
    ids = torch.from_numpy(gen.randint(1604, (3, 17), 0, 20))
    with torch.no_grad():
        lg = d(ids)
        cl = d(ids, generate=False)
    save("ref_ckpt_outputs.npz", vq_x_hat=xh.numpy(), vq_emb_loss=e.numpy(), vq_perplexity=p.numpy(),
         vq_idx=idx.view(-1).numpy().astype(np.int64), dec_logits=lg.numpy(), dec_class_logits=cl.numpy())


def main(only=()):
    """python tests/golden/make_golden.py [case ...]: every case, or only the named ones (vq_small vq_idx vqvae
    decoder radam regime asimow ckpt)."""
    install_shim()
    torch.set_num_threads(8)
    from model.vector_quantizer import VectorQuantizer
    from model.vq_vae_patch_embedd import VQVAEPatch
    from model.transformer_decoder import MyTransformerDecoder
    cases = {"vq_small": lambda: case_vq_small(VectorQuantizer), "vq_idx": lambda: case_vq_idx(VectorQuantizer),
             "vqvae": lambda: case_vqvae(VQVAEPatch), "decoder": lambda: case_decoder(MyTransformerDecoder),
             "radam": case_radam, "regime": lambda: case_training_regime(MyTransformerDecoder),
             "asimow": case_asimow, "ckpt": lambda: case_checkpoints(VQVAEPatch, MyTransformerDecoder)}
    for name, fn in cases.items():
        if not only or name in only:
            fn()


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
