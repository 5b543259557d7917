"""The real data-parallel path on the GPU: two ranks over gloo sharing cuda:0 (RCCL refuses two
ranks on one device; the collective calls are the same), each running Trainer.graphed_step -- the captured step
graphs, the bucketed all-reduce of the live spans of the flat gradient buffer (the VQ-VAE's dead encoder side taps
left out), the VQ-VAE's split late/early all-reduce around the decoder-side backward, the decoder's per-block
overlapped buckets -- and Trainer.optimizer_step on the real models.

Reference (DDP semantics, no SyncBN): each optimizer step uses the mean of the two ranks' gradients, each rank's
gradient taken on its own half batch (BatchNorm statistics per rank) -- computed here in one process as
accumulate 2 x scale 1/2 on the two halves in turn.  After the steps every rank's parameters equal the
reference's.  Dropout is 0 so that both sides draw no masks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import decoder as od
from oracle import gen
from oracle import vqvae as ov

pytestmark = pytest.mark.gpu

VQ_KW = dict(hidden_dim=64, num_embeddings=64, embedding_dim=16, n_resblocks=2, patch_size=25)
DEC_KW = dict(d_model=64, n_classes=34, seq_len=33, n_blocks=3)
STEPS = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _vqvae():
    from model.vq_vae_patch_embedd import VQVAEPatch
    m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, **VQ_KW)
    sd = ov.det_state_dict(ov.VQVAEConfig(**VQ_KW), 1901)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def _decoder():
    from model.transformer_decoder import MyTransformerDecoder
    m = MyTransformerDecoder(n_head=4, res_dropout=0.0, att_dropout=0.0, **DEC_KW)
    sd = od.det_state_dict(1902, **DEC_KW)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def _vq_batches():
    return [torch.tensor(gen.windows(1910 + s, 16)) for s in range(STEPS)]


def _dec_batches():
    out = []
    for s in range(STEPS):
        ids = torch.tensor(gen.randint(1920 + s, (8, DEC_KW["seq_len"] + 1), 0, DEC_KW["n_classes"] - 2))
        out.append((ids[:, :-1].contiguous(), torch.zeros(8, dtype=torch.long), ids[:, 1:].contiguous()))
    return out


def _half(batch, r, world):
    if isinstance(batch, torch.Tensor):
        n = batch.shape[0] // world
        return batch[r * n:(r + 1) * n].cuda()
    return tuple(_half(b, r, world) for b in batch)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    try:
        with operands(torch.float32):
            for name, make, batches in (("vqvae", _vqvae, _vq_batches()), ("decoder", _decoder, _dec_batches())):
                m = make()
                if rank == 1:       # the initial broadcast must replace rank 1's parameters
                    with torch.no_grad():
                        for p in m.parameters():
                            p.add_(0.5)
                tr = Trainer(gradient_clip_val=0.7 if name == "vqvae" else 0.8)
                tr.setup_optimizer(m)
                for s, b in enumerate(batches):
                    hb = _half(b, rank, world)
                    if s == 0:      # one eager step; then graphed_step: two eager warm-up calls, capture, replay
                        tr.micro_step(m, hb, 0, 1.0 / world)
                        tr.optimizer_step(m)
                    else:
                        tr.graphed_step(m, hb, 1.0 / world)
                torch.cuda.synchronize()
                out[(name, rank)] = {k: v.detach().cpu().clone() for k, v in m.named_parameters()}
    finally:
        dist.destroy_process_group()


def _reference(name, make, batches):
    """One process: per step, micro-batches = the two ranks' halves, loss scale 1/2 each (gradient mean)."""
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    with operands(torch.float32):
        m = make()
        tr = Trainer(gradient_clip_val=0.7 if name == "vqvae" else 0.8, accumulate_grad_batches=2)
        tr.setup_optimizer(m)
        for b in batches:
            for r in range(2):
                tr.micro_step(m, _half(b, r, 2), r, 0.5)
            tr.optimizer_step(m)
        torch.cuda.synchronize()
        return {k: v.detach().cpu().clone() for k, v in m.named_parameters()}


def test_data_parallel_world2_matches_gradient_mean_reference():
    port = _free_port()
    # the manager's server process is spawned, not forked: a fork of this process (which may already hold the GPU
    # from earlier tests) can crash in the child's garbage collector
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    for name, make, batches in (("vqvae", _vqvae, _vq_batches()), ("decoder", _decoder, _dec_batches())):
        ref = _reference(name, make, batches)
        for r in range(2):
            got = out[(name, r)]
            for k, v in ref.items():
                torch.testing.assert_close(got[k], v, rtol=1e-5, atol=1e-6, msg=f"{name} rank {r} {k}")
        # the ranks moved away from the initial weights (the steps did something)
        init = make()
        moved = [k for k, v in init.named_parameters() if not torch.equal(v.detach().cpu(), ref[k])]
        assert len(moved) > len(ref) // 2, name
        np.testing.assert_equal(sorted(out[(name, 0)]), sorted(ref))
