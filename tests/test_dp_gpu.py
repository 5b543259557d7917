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


# ------------------------------------------------------------------------------------------------ full size
# configs[3]'s per-rank workload shape (train_transformer_mtasks.py:31,87,149-153): the VQ-VAE at
# H512 / R8 / K512xD64 and the 8-block d512 decoder at T = 257 (16 cycles of 16 tokens + 1).  At these sizes the
# live gradient spans are tens of MB, so the bucketed all-reduce issues several buckets per region: the decoder
# ~50 MB per region at the default 32 MiB buckets, the VQ-VAE's late (decoder-side) region 56 MB; its early region
# (patch embed + the 16 encoder centre taps + sep conv, 17 MB) fits one default bucket, so a second VQ-VAE run uses
# 4 MiB buckets to cut every region into many buckets at offsets that are not segment boundaries.
FULL_VQ = dict(hidden_dim=512, num_embeddings=512, embedding_dim=64, n_resblocks=8, patch_size=25)
FULL_DEC = dict(d_model=512, n_classes=514, seq_len=257, n_blocks=8)
FULL_RUNS = (("vqvae", 8 * 1024 * 1024), ("vqvae", 1024 * 1024), ("decoder", 8 * 1024 * 1024))


def _full_make(name):
    if name == "vqvae":
        from model.vq_vae_patch_embedd import VQVAEPatch
        m = VQVAEPatch(input_dim=2, learning_rate=1e-3, dropout_p=0.0, batch_norm=False, **FULL_VQ)
        sd = ov.det_state_dict(ov.VQVAEConfig(**FULL_VQ), 1931)
    else:
        from model.transformer_decoder import MyTransformerDecoder
        m = MyTransformerDecoder(n_head=8, res_dropout=0.0, att_dropout=0.0, **FULL_DEC)
        sd = od.det_state_dict(1932, **FULL_DEC)
    m.load_state_dict({k: torch.tensor(v) for k, v in sd.items()})
    return m.cuda().train()


def _full_batches(name):
    if name == "vqvae":
        return [torch.tensor(gen.windows(1940 + s, 256)) for s in range(STEPS)]
    out = []
    for s in range(STEPS):
        ids = torch.tensor(gen.randint(1950 + s, (16, FULL_DEC["seq_len"] + 1), 0, FULL_DEC["n_classes"] - 2))
        out.append((ids[:, :-1].contiguous(), torch.zeros(16, dtype=torch.long), ids[:, 1:].contiguous()))
    return out


def _full_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from arcweld.precision import operands
    from arcweld.trainer import Trainer
    sizes = []
    orig_ar = dist.all_reduce

    def counting_all_reduce(t, *a, **kw):
        sizes.append(t.numel())
        return orig_ar(t, *a, **kw)

    dist.all_reduce = counting_all_reduce
    try:
        with operands(torch.float32):
            for run, (name, bucket) in enumerate(FULL_RUNS):
                m = _full_make(name)
                tr = Trainer(gradient_clip_val=0.7 if name == "vqvae" else 0.8)
                tr.bucket_elems = bucket
                tr.setup_optimizer(m)
                regions = []
                orig_region = tr._allreduce_region

                def rec(model, region, _orig=orig_region, _log=regions):
                    n0 = len(sizes)
                    works = _orig(model, region)
                    _log.append((region, sizes[n0:]))
                    return works

                tr._allreduce_region = rec
                for s, b in enumerate(_full_batches(name)):
                    hb = _half(b, rank, world)
                    if s == 0:
                        tr.micro_step(m, hb, 0, 1.0 / world)
                        tr.optimizer_step(m)
                    else:
                        tr.graphed_step(m, hb, 1.0 / world)
                torch.cuda.synchronize()
                live = sum(b - a for a, b in tr.optimizer.live_spans())
                out[(run, rank)] = dict(params={k: v.detach().cpu().clone() for k, v in m.named_parameters()},
                                        regions=regions, live=live)
                del m, tr
                torch.cuda.empty_cache()
    finally:
        dist.all_reduce = orig_ar
        dist.destroy_process_group()


def test_data_parallel_world2_full_size_multi_bucket():
    port = _free_port()
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_full_worker, args=(2, port, out), nprocs=2, join=True)
    for run, (name, bucket) in enumerate(FULL_RUNS):
        ref = _reference(name, lambda: _full_make(name), _full_batches(name))
        for r in range(2):
            got = out[(run, r)]
            for k, v in ref.items():
                torch.testing.assert_close(got["params"][k], v, rtol=1e-5, atol=1e-6,
                                           msg=f"{name} bucket {bucket} rank {r} {k}")
            split = [(reg, sz) for reg, sz in got["regions"] if reg in ("late", "early")]
            assert split, "the captured step never took the late/early split all-reduce"
            for reg, sz in split:
                assert max(sz) <= bucket and sum(sz) > 0, (name, reg, sz)
                if not (name == "vqvae" and reg == "early" and bucket == 8 * 1024 * 1024):
                    assert len(sz) > 1, f"{name}: region {reg} issued one bucket at {bucket} elements"
            # one replayed step reduces every live gradient once, split between the two regions (the late set's
            # merged spans may carry the <= 63-element alignment padding between its adjacent segments)
            late, early = split[-2][1], split[-1][1]
            tot = sum(late) + sum(early)
            assert got["live"] <= tot <= got["live"] + 64 * len(ref), (name, sum(late), sum(early), got["live"])
